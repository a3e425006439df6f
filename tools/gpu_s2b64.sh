#!/bin/bash
# 64-input-channel stride-2 halo backward-data: tests, then conv_bench off / on
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 300 ktest python3 -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "s2bwd or fast_path or staged or ragged"
SH=c4x4s2_64_128,c4x4s2_32_256
step 200 s0 env EEGAN_CONV_S2B64=0 python3 tools/conv_bench.py --shapes $SH --dirs bwdd --device-time
step 200 s1 python3 tools/conv_bench.py --shapes $SH --dirs bwdd --device-time
paste <(grep -h 'us ' gpurun_out/s0.log) <(grep -h 'us ' gpurun_out/s1.log | cut -c18-)
