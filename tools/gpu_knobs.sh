#!/bin/bash
# Planner knob sweep on the real step (graph replay): one bench line per setting.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KNOBS=${KNOBS:-"base EEGAN_CONV=target=256 EEGAN_CONV=target=1024 EEGAN_CONV=wgrad_target=256 EEGAN_CONV=wgrad_target=1024 EEGAN_CONV=mink=8 EEGAN_CONV=mink=32 EEGAN_CONV=wgrad_minp=256 EEGAN_CONV=wgrad_minp=1024 base"}
for kv in $KNOBS; do
  if [ $kv = base ]; then e=""; else e="$kv"; fi
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 30 > gpurun_out/knob.log 2>&1 || exit 1
  echo "$kv $(grep -h '"metric"' gpurun_out/knob.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
