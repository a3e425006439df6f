#!/bin/bash
# Planner knob sweep on the real step (graph replay): one bench line per setting.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KNOBS=${KNOBS:-"base EEGAN_CONV_TARGET=256 EEGAN_CONV_TARGET=1024 EEGAN_WGRAD_TARGET=256 EEGAN_WGRAD_TARGET=1024 EEGAN_CONV_MINK=8 EEGAN_CONV_MINK=32 EEGAN_WGRAD_MINP=256 EEGAN_WGRAD_MINP=1024 base"}
for kv in $KNOBS; do
  if [ $kv = base ]; then e=""; else e="${kv//,/ }"; fi
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 30 > gpurun_out/knob.log 2>&1 || exit 1
  echo "$kv $(grep -h '"metric"' gpurun_out/knob.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
