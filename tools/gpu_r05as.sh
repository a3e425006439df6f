#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05as}
step 400 ${TAG}_C3 python3 bench.py --config C3 --no-cpu-baseline --steps 10
grep -h '"metric"' gpurun_out/${TAG}_C3.log | cut -c1-200
step 300 ${TAG}_C2_20 python3 bench.py --no-cpu-baseline --steps 20
grep -h '"metric"' gpurun_out/${TAG}_C2_20.log | cut -c1-200
