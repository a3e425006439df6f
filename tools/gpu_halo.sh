#!/bin/bash
# halo 3x3 kernel: the conv kernel tests, conv_bench of the 3x3 shapes, per-shape conv time of the step,
# in-process A/B of the replayed step
source ./run_gpu_steps.sh
TAG=${1:-halo}
S=c3x3_64_128,c3x3_128_64,c3x3_256_32,d256_b0_3x3,d256_b1_3x3,d256_b2_3x3
step 300 ${TAG}_ktests python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread
step 200 ${TAG}_gen python3 -u -m pytest tests/test_gpu_models.py -x -q -s -k "test_generator" --timeout 120 --timeout-method thread
step 200 ${TAG}_cb python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd --device-time
step 200 ${TAG}_shapes python3 tools/conv_shapes.py --top 400
step 400 ${TAG}_ab python3 tools/ab_inproc.py EEGAN_CONV=halo=0 --reps 4 --steps 20
tail -2 gpurun_out/${TAG}_ab.log
