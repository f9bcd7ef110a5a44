tools/gpu_step.sh \
 "400 kt15.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "300 bench15.log python bench.py --steps 20 --warmup 5"
