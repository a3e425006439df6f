#!/bin/bash
# Process-level A/B of EEGAN_LANE_PRIO (read when the lanes are created, so not switchable in-process)
source ./run_gpu_steps.sh
for i in 1 2 3 4; do
  for p in 1 2 0; do
    EEGAN_LANE_PRIO=$p step 300 lp_${p}_$i python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timer || exit $?
  done
done
for p in 1 2 0; do echo "LANE_PRIO=$p: $(grep -h '"metric"' gpurun_out/lp_${p}_*.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["value"]) for l in sys.stdin))')"; done
