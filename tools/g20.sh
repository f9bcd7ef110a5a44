tools/gpu_step.sh \
 "900 gputests_final.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 smoke_final.log python -c 'import __graft_entry__ as g; g.smoke()'"
