#!/bin/bash
# Bench A/B of an environment switch: alternating runs, graph replay, no timing pass.
#   bash tools/gpu_ab_env.sh "EEGAN_STREAMS=0" [reps] [extra bench args]
cd "$GRAFT_REPO_ROOT"
ENVB=$1; REPS=${2:-3}; shift; shift
for i in $(seq $REPS); do
  a=$(timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-timer --steps 30 "$@" | grep -o '"value": [0-9.]*') || exit 1
  b=$(env $ENVB timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-timer --steps 30 "$@" | grep -o '"value": [0-9.]*') || exit 1
  echo "A (default) $a    B ($ENVB) $b"
done
