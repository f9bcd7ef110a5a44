tools/gpu_step.sh \
 "300 kt.log python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'conv or gemm'" \
 "300 tw_k2.log python tools/tune_conv.py --batch 256 --knob 2 --values 0,1 --pass wgrad" \
 "300 tw_k3.log python tools/tune_conv.py --batch 256 --knob 3 --values 0,1,2 --pass wgrad --set 2=1" \
 "300 tw_k3m1.log python tools/tune_conv.py --batch 256 --knob 3 --values 0,1,2 --pass wgrad --set 2=1,0=1"
