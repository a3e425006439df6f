#!/bin/bash
# A/B of lane issue order and hardware queue count: phase timeline + bench line per setting.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
for v in "fwd 4" "rev 4" "fwd 8" "rev 8"; do
  set -- $v
  step 300 lane_$1_q$2 env EEGAN_LANE_ORDER=$1 GPU_MAX_HW_QUEUES=$2 python3 -u tools/stamp_phases.py
  step 300 lanebench_$1_q$2 env EEGAN_LANE_ORDER=$1 GPU_MAX_HW_QUEUES=$2 python3 bench.py --no-cpu-baseline --no-timer --steps 20
done
for f in gpurun_out/lanebench_*.log; do echo $f; grep -h '"metric"' $f | cut -c1-200; done
for f in gpurun_out/lane_*.log; do echo $f; grep -E "step \(start|D2 start|DAMSM backward|D2 gp adam" $f; done
