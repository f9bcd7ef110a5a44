tools/gpu_step.sh \
 "300 t_acc.log python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'stacked or bottleneck or resnet' -s"
