#!/bin/bash
# split-K fused finish stress; FORCE_DIST captured comm lanes; C2 graph==eager (fused, twice)
source ./run_gpu_steps.sh
TAG=${1:-r05f}
step 300 ${TAG}_stress python3 tools/splitk_stress.py --iters 300
mkdir -p gpurun_out/fd
step 300 ${TAG}_fd_lane env EEGAN_FORCE_DIST=1 DP_COMM_LANES=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29552 tools/with_bt.py tests/dp_force_worker.py gpurun_out/fd lane graph
step 300 ${TAG}_c2a python3 -u -m pytest tests/test_gpu_models.py -x -q -s -k "test_config_step_graph_matches_eager and C2" --timeout 250 --timeout-method thread
step 300 ${TAG}_c2b python3 -u -m pytest tests/test_gpu_models.py -x -q -s -k "test_config_step_graph_matches_eager and C2" --timeout 250 --timeout-method thread
grep -h "splitk stress" gpurun_out/${TAG}_stress.log
grep -h "STEPGRAPH\|passed\|failed" gpurun_out/${TAG}_c2*.log
tail -5 gpurun_out/${TAG}_fd_lane.log
