#!/bin/bash
# conv_bench of the 3x3 halo shapes: tools/ab_lib/libeegan_hip_base.so vs the in-tree
# library (and tools/ab_lib/libeegan_hip_$LIBS.so, and in-tree with EEGAN_CONV variants in $VARS),
# same box, two rounds
source ./run_gpu_steps.sh
TAG=${1:-hab}
S=${S:-c3x3_64_128,c3x3_128_64,c3x3_256_32,d256_b0_3x3,d256_b1_3x3,d256_b2_3x3}
for r in 1 2; do
  step 200 ${TAG}_base_$r env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_base.so python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd --device-time
  step 200 ${TAG}_new_$r python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd --device-time
  for l in $LIBS; do
    step 200 ${TAG}_${l}_$r env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_$l.so python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd --device-time
  done
  for v in $VARS; do
    step 200 ${TAG}_${v}_$r env EEGAN_CONV=$v python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd --device-time
  done
done
for f in gpurun_out/${TAG}_*.log; do echo "== $f"; grep -h 'TF/s' $f; done
