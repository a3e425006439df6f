#!/bin/bash
# BN kernels: bn_bench (in-tree vs tools/ab_lib base), BN / generator / step tests
source ./run_gpu_steps.sh
TAG=${1:-bn5}
step 200 ${TAG}_base env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_base.so python3 tools/bn_bench.py
step 200 ${TAG}_new python3 tools/bn_bench.py
step 400 ${TAG}_tests python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "bn or BN or generator or syncbn or sagb or cum or step_graph" --timeout 200 --timeout-method thread
grep -h "bwd reduce" gpurun_out/${TAG}_base.log gpurun_out/${TAG}_new.log
