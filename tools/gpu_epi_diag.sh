#!/bin/bash
# tile-kernel epilogue: bit-identity of the LDS-staged form, then conv_bench
# with direct (EEGAN_CONV_STAGE_EPI=0) / staged / knocked-out (EEGAN_CONV_NOLOAD=4) epilogues
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 300 ktest python3 -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "staged_epilogue or s2bwd or 1x1 or wide_stages or fast_path or conv_fwd_bwd or double_backward"
SH=c3x3_64_128,c3x3_128_64,c3x3_256_32,c3x3_512_16,c4x4s2_128_64,c4x4s2_32_256,c3x3_32_256
step 200 epi0 env EEGAN_CONV_STAGE_EPI=0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
step 200 epi1 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
step 200 epi4 env EEGAN_CONV_NOLOAD=4 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd --device-time
paste <(grep -h 'us ' gpurun_out/epi0.log) <(grep -h 'us ' gpurun_out/epi1.log | cut -c18-) <(grep -h 'us ' gpurun_out/epi4.log | cut -c18-)
