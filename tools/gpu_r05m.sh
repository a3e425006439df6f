#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05m}
step 300 ${TAG}_bnr4 env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_bnr4.so python3 tools/determinism.py --config C2 --reps 14 --steps 1
step 300 ${TAG}_head python3 tools/determinism.py --config C2 --reps 14 --steps 1
for f in bnr4 head; do echo "== $f"; grep -h "determinism" gpurun_out/${TAG}_$f.log | grep -vc "G 0.000e+00/0.000e+00  D0 0.000e+00/0.000e+00  D1 0.000e+00/0.000e+00  D2 0.000e+00/0.000e+00"; done
