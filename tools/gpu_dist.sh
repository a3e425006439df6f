#!/bin/bash
# Multi-rank rehearsals on a one-GPU box: (1) one rank with every collective
# issued through the own-RCCL communicators and captured in the step graph,
# (2) two ranks sharing the GPU over gloo (eager).
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 600 force_dist env EEGAN_FORCE_DIST=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline
grep -h '"metric"' gpurun_out/force_dist.log
step 700 dp2 bash tools/rehearse_dp2.sh
grep -h '"metric"' gpurun_out/dp2.log
