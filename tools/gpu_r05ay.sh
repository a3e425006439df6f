#!/bin/bash
# 64-channel output tiles of the halo weight gradient: parity, conv_bench, in-process A/B
source ./run_gpu_steps.sh
TAG=${1:-r05ay}
step 400 ${TAG}_tests python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad"
SH=d256_b0_3x3,c3x3_64_128,c3x3_32_256,c3x3_64_32_256,d256_b1_3x3,c3x3_128_64
step 300 ${TAG}_cb1 python3 tools/conv_bench.py --shapes $SH --dirs wgrad
step 300 ${TAG}_cb0 env EEGAN_CONV=wgrad_halo_cot64=0 python3 tools/conv_bench.py --shapes $SH --dirs wgrad
for f in gpurun_out/${TAG}_cb*.log; do echo "== $f"; grep -E "TF/s" $f; done
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=wgrad_halo_cot64=0" --reps 4 --steps 20
tail -3 gpurun_out/${TAG}_ab.log
