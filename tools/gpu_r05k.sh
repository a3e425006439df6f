#!/bin/bash
# determinism bisect: head / r4 BN kernels / unfused split-K / no GEN_SIDE
source ./run_gpu_steps.sh
TAG=${1:-r05k}
step 300 ${TAG}_head python3 tools/determinism.py --config C2 --reps 6 --steps 2
step 300 ${TAG}_bnr4 env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_bnr4.so python3 tools/determinism.py --config C2 --reps 6 --steps 2
step 300 ${TAG}_nofuse env EEGAN_CONV=splitk_fused=0 python3 tools/determinism.py --config C2 --reps 6 --steps 2
step 300 ${TAG}_noside python3 -c "
import sys; sys.argv=['x','--config','C2','--reps','6','--steps','2']
sys.path[:0]=['ee-gan_amd','.']
import eegan_hip.trainer as TR; TR.GEN_SIDE=False
import runpy; runpy.run_path('tools/determinism.py', run_name='__main__')"
for f in head bnr4 nofuse noside; do echo "== $f"; grep -h "determinism" gpurun_out/${TAG}_$f.log | cut -c1-140; done
