#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05n}
step 300 ${TAG}_br python3 tools/gen_determinism.py --reps 25
step 300 ${TAG}_single python3 tools/gen_determinism.py --reps 25 --single
step 300 ${TAG}_br_bnr4 env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_bnr4.so python3 tools/gen_determinism.py --reps 25
grep -h "gen determinism" gpurun_out/${TAG}_*.log | cut -c1-300
