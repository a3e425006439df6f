#!/bin/bash
# DREAL_EARLY lane placement A/B
source ./run_gpu_steps.sh
TAG=${1:-r05y}
step 600 ${TAG}_tests python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "real_early"
for v in none 2:own 2:damsm 1,2:own 1,2:damsm none; do
  e=${v%%:*}; l=${v##*:}; [ "$v" = none ] && e= && l=own
  step 300 ${TAG}_bench_$v env EEGAN_DREAL_EARLY=$e EEGAN_DREAL_LANE=$l python3 bench.py --no-cpu-baseline --steps 20
  echo "$v: $(grep -ho '"value": [0-9.]*' gpurun_out/${TAG}_bench_$v.log)"
done
step 300 ${TAG}_phases_own env EEGAN_DREAL_EARLY=2 EEGAN_DREAL_LANE=own python3 -u tools/stamp_phases.py
step 300 ${TAG}_phases_damsm env EEGAN_DREAL_EARLY=2 EEGAN_DREAL_LANE=damsm python3 -u tools/stamp_phases.py
