#!/bin/bash
# DREAL_EARLY: tests + A/B bench lines
source ./run_gpu_steps.sh
TAG=${1:-r05x}
step 600 ${TAG}_tests python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "real_early or full_step or graph_matches_eager or deterministic"
for v in 2 none 1,2 0,1,2; do
  e=$v; [ "$v" = none ] && e=
  step 300 ${TAG}_bench_$v env EEGAN_DREAL_EARLY=$e python3 bench.py --no-cpu-baseline --steps 20
done
for v in 2 none 1,2 0,1,2; do echo "$v: $(grep -ho '"value": [0-9.]*' gpurun_out/${TAG}_bench_$v.log)"; done
step 300 ${TAG}_phases python3 -u tools/stamp_phases.py
