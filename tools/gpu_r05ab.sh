#!/bin/bash
# halo3r with the pinned MFMA / LDS-read schedule: conv_bench A/B + tpb sweep + step A/B
source ./run_gpu_steps.sh
TAG=${1:-r05ab}
step 400 ${TAG}_tests python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "halo3r"
SH=d256_b0_3x3,c3x3_64_128
step 300 ${TAG}_cb_r0 env EEGAN_CONV=halo_r=0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd
for t in 0 2 4 8 16; do
  step 300 ${TAG}_cb_tpb$t env EEGAN_CONV=halo_r_tpb=$t python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd
done
for f in gpurun_out/${TAG}_cb_*.log; do echo "== $f"; grep -E "TF/s" $f; done
