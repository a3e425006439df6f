#!/bin/bash
# diagnose: C2 graph==eager with and without the fused split-K finish; FORCE_DIST graph segfault backtrace
source ./run_gpu_steps.sh
TAG=${1:-r05e}
step 300 ${TAG}_c2_nofuse env EEGAN_CONV=splitk_fused=0 python3 -u -m pytest tests/test_gpu_models.py -x -q -s -k "test_config_step_graph_matches_eager and C2" --timeout 250 --timeout-method thread
step 300 ${TAG}_c2_fuse python3 -u -m pytest tests/test_gpu_models.py -x -q -s -k "test_config_step_graph_matches_eager and C2" --timeout 250 --timeout-method thread
mkdir -p gpurun_out/fd
step 300 ${TAG}_fd_inlane env EEGAN_FORCE_DIST=1 DP_COMM_LANES=0 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 tests/dp_force_worker.py gpurun_out/fd inlane graph
step 300 ${TAG}_fd_lane env EEGAN_FORCE_DIST=1 DP_COMM_LANES=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29552 tools/with_bt.py tests/dp_force_worker.py gpurun_out/fd lane graph
grep -h "STEPGRAPH\|passed\|failed" gpurun_out/${TAG}_c2_*.log
tail -40 gpurun_out/${TAG}_fd_lane.log | grep -v "^\s*$" | tail -30
