#!/bin/bash
# A/B of the stride-2 halo backward-data and 1x1 streaming conv kernels:
# bit-identity tests, then conv_bench device time with each path off / on.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 300 ktest python3 -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "s2bwd or 1x1 or fast_path or wide_stages or splitk or conv_fwd_bwd or double_backward"
SH=c4x4s2_32_256,c1x1_32_128,c1x1_32_256,c1x1_64_64,c1x1_128_32,c1x1_256_4,c1x1_100_128
step 200 cb0 env EEGAN_CONV_S2B=0 EEGAN_CONV_1X1=0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
step 200 cb1 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
grep -h -v Warn gpurun_out/cb0.log gpurun_out/cb1.log
