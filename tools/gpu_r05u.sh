#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05u}
for i in 1 2; do
  step 300 ${TAG}_oldDX_$i env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_oldDX.so python3 tools/gen_determinism.py --reps 40 --load
  step 300 ${TAG}_head_$i python3 tools/gen_determinism.py --reps 40 --load
  step 300 ${TAG}_nofuse_$i env EEGAN_CONV=splitk_fused=0 python3 tools/gen_determinism.py --reps 40 --load
done
for f in gpurun_out/${TAG}_*.log; do echo "$f: $(grep -h 'repetitions differ' $f)"; done
