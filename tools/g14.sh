tools/gpu_step.sh "200 arena.log python tools/arena_check.py"
