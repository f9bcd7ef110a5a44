tools/gpu_step.sh \
 "300 tdx_t.log python tools/tune_conv.py --batch 256 --knob 4 --values 0,1,2,3,4 --pass dx" \
 "300 tfw_t.log python tools/tune_conv.py --batch 256 --knob 4 --values 0,1,2,3,4 --pass fwd"
