#!/bin/bash
# halo3r knock-outs (timing only): 1 = no halo loads after the first tile, 2 = no epilogue
source ./run_gpu_steps.sh
TAG=${1:-r05ac}
SH=d256_b0_3x3,c3x3_64_128
for k in 0 1 2 3; do
  step 300 ${TAG}_k$k env EEGAN_CONV=halo_r_tpb=16,halo_r_knock=$k python3 tools/conv_bench.py --shapes $SH --dirs fwd
done
for f in gpurun_out/${TAG}_k*.log; do echo "== $f"; grep -E "TF/s" $f; done
