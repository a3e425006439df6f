#!/bin/bash
# ragged-channel (C % 8 != 0) LDS-DMA path: tests, then conv_bench register-staged vs LDS-DMA
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 300 ktest python3 -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "ragged or fast_path or conv_fwd_bwd or double_backward or staged or wide"
SH=c3x3_64_100_128,c3x3_128_100_64
step 200 g0 env EEGAN_CONV_GLDS_RAGGED=0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
step 200 g1 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
paste <(grep -h 'us ' gpurun_out/g0.log) <(grep -h 'us ' gpurun_out/g1.log | cut -c18-)
