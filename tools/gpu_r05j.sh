#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05j}
step 300 ${TAG}_det python3 tools/determinism.py --config C2 --reps 8 --steps 2
step 400 ${TAG}_tests python3 -u -m pytest tests/test_gpu_models.py -x -q -s -k "deterministic or step_graph" --timeout 250 --timeout-method thread
grep -h "determinism" gpurun_out/${TAG}_det.log
grep -h "DETERMINISM\|STEPGRAPH\|passed\|failed" gpurun_out/${TAG}_tests.log
