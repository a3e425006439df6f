#!/bin/bash
# BN kernel A/B + tests; the data-parallel tests (comm lanes, FORCE_DIST capture)
source ./run_gpu_steps.sh
TAG=${1:-r05c}
step 200 ${TAG}_bnbase env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_base.so python3 tools/bn_bench.py
step 200 ${TAG}_bnnew python3 tools/bn_bench.py
step 500 ${TAG}_bntests python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "bn or BN or generator or syncbn or sagb or cum or step_graph" --timeout 200 --timeout-method thread
step 600 ${TAG}_dist python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_peer.py -x -v -s --timeout 300 --timeout-method thread
grep -h "bwd reduce" gpurun_out/${TAG}_bnbase.log gpurun_out/${TAG}_bnnew.log
tail -3 gpurun_out/${TAG}_bntests.log
grep -E "PASSED|FAILED|Error|overlap:|FORCE" gpurun_out/${TAG}_dist.log | head
