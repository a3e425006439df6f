#!/bin/bash
# halo3r with the fragment epilogue: parity, conv_bench A/B + tpb sweep, step A/B
source ./run_gpu_steps.sh
TAG=${1:-r05ad}
step 400 ${TAG}_tests python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "halo3"
SH=d256_b0_3x3,c3x3_64_128
step 300 ${TAG}_cb_r0 env EEGAN_CONV=halo_r=0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd
for t in 0 4 8 16; do
  step 300 ${TAG}_cb_tpb$t env EEGAN_CONV=halo_r_tpb=$t python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd
done
step 300 ${TAG}_cb_k2 env EEGAN_CONV=halo_r_tpb=16,halo_r_knock=2 python3 tools/conv_bench.py --shapes $SH --dirs fwd
for f in gpurun_out/${TAG}_cb_*.log; do echo "== $f"; grep -E "TF/s" $f; done
for r in 1 2; do
  step 300 ${TAG}_b_r1_$r python3 bench.py --no-cpu-baseline --steps 20
  step 300 ${TAG}_b_r0_$r env EEGAN_CONV=halo_r=0 python3 bench.py --no-cpu-baseline --steps 20
done
for v in r1 r0; do echo "$v: $(grep -ho '"value": [0-9.]*' gpurun_out/${TAG}_b_${v}_1.log) $(grep -ho '"value": [0-9.]*' gpurun_out/${TAG}_b_${v}_2.log)"; done
