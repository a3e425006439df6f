#!/bin/bash
# bench.py lines (no cpu baseline / timer) for env settings, ROUNDS rotations:
#   SETTINGS="base EEGAN_LANE_PRIO=2 ..." (commas join several vars in one setting)
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
SETTINGS=${SETTINGS:-"base"}
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for kv in $SETTINGS; do
    if [ $kv = base ]; then e=""; else e="${kv//,/ }"; fi
    tag=$(echo "$kv" | tr '=,' '__')
    step 300 envab_${tag}_$r env $e python3 bench.py --no-cpu-baseline --no-timer --steps 20
    echo "$kv round $r: $(grep -h '"metric"' gpurun_out/envab_${tag}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
