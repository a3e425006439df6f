#!/bin/bash
# Wide (64-channel) conv stages: bit-identity tests, then conv_bench with and without.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
SH=${1:-c3x3_64_128,c3x3_128_64,c3x3_256_32,c3x3_512_16,c4x4s2_128_64,c4x4s2_512_8,c3x3_512_8,c1x1_768_17,c4x4s2_32_256}
step 300 widetest python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or splitk or conv" || exit 1
grep -q "failed" gpurun_out/widetest.log && exit 1
EEGAN_CONV_WIDE=0 step 200 cw0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
EEGAN_CONV_WIDE=1 step 200 cw1 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
paste <(grep -v amdgpu gpurun_out/cw0.log) <(grep -v amdgpu gpurun_out/cw1.log | awk '{print $3, $4, $5, $6}')
