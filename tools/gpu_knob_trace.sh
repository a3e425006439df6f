#!/bin/bash
# Planner knobs judged by summed kernel time per step (rocprofv3 kernel trace of
# the bench's graph replays) instead of img/s, which varies ~6% between
# processes.  KNOBS="base EEGAN_CONV_MINK=32 ..." (commas separate several vars).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KNOBS=${KNOBS:-"base EEGAN_CONV_MINK=32 base"}
i=0
for kv in $KNOBS; do
  i=$((i + 1))
  if [ $kv = base ]; then e=""; else e="${kv//,/ }"; fi
  d=gpurun_out/kt_$i
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-timer > gpurun_out/kt_$i.log 2>&1 || exit 1
  echo "$kv $(python3 tools/dispatch_groups.py $d --steps 22 --top 3 --by-name | head -1) \
$(grep -h '"metric"' gpurun_out/kt_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  find $d -name '*.csv' -delete
done
