#!/bin/bash
# lane gating A/B (EEGAN_LANE_GATE), two rounds
source ./run_gpu_steps.sh
TAG=${1:-r05z}
V="none 0:2:loss 0:2:adam,1:2:adam 0:2:loss,1:2:loss 0:2:gp 1:2:loss 0:1:gp"
for r in 1 2; do
for v in $V; do
  e=$v; [ "$v" = none ] && e=
  step 300 ${TAG}_${v}_$r env EEGAN_LANE_GATE=$e python3 bench.py --no-cpu-baseline --steps 20
done
done
for v in $V; do echo "$v: $(grep -ho '"value": [0-9.]*' gpurun_out/${TAG}_${v}_1.log) $(grep -ho '"value": [0-9.]*' gpurun_out/${TAG}_${v}_2.log)"; done
