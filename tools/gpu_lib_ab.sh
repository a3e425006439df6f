#!/bin/bash
# A/B of two builds of the library on the replayed step: tools/ab_lib/libeegan_hip_base.so
# (the previous build) against the in-tree one, ROUNDS rotations of bench.py (20 steps).
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for v in base new; do
    if [ $v = base ]; then e="EEGAN_HIP_LIB=$GRAFT_REPO_ROOT/tools/ab_lib/libeegan_hip_base.so"; else e=""; fi
    step 300 libab_${v}_$r env $e python3 bench.py --no-cpu-baseline --no-timer --steps ${STEPS:-20}
    echo "$v round $r: $(grep -h '"metric"' gpurun_out/libab_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
