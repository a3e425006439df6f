#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05v}
for i in 1 2 3; do
  step 300 ${TAG}_head_$i python3 tools/gen_determinism.py --reps 40 --load
done
for f in gpurun_out/${TAG}_head_*.log; do echo "$f: $(grep -h 'repetitions differ' $f)"; done
step 600 ${TAG}_tests python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "deterministic or graph_matches_eager or branched"
