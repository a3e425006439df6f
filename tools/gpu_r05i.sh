#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05i}
step 300 ${TAG}_det python3 tools/determinism.py --config C2 --reps 6 --steps 2
step 400 ${TAG}_tests python3 -u -m pytest tests/test_gpu_models.py -x -q -s -k "deterministic or step_graph or full_step or branched" --timeout 250 --timeout-method thread
step 600 ${TAG}_dist python3 -u -m pytest tests/test_gpu_dist.py -x -q -s --timeout 300 --timeout-method thread
step 300 ${TAG}_bench python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
grep -h "determinism" gpurun_out/${TAG}_det.log
grep -h "DETERMINISM\|STEPGRAPH\|passed\|failed" gpurun_out/${TAG}_tests.log gpurun_out/${TAG}_dist.log
grep -h '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-200
