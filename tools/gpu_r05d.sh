#!/bin/bash
# BN kernel A/B, kernel tests (split-K fused finish), dist tests, bench line
source ./run_gpu_steps.sh
TAG=${1:-r05d}
step 200 ${TAG}_bnbase env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_base.so python3 tools/bn_bench.py
step 200 ${TAG}_bnnew python3 tools/bn_bench.py
step 600 ${TAG}_ktests python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread
step 600 ${TAG}_gen python3 -u -m pytest tests/test_gpu_models.py -x -q -k "generator or sagb or cum or syncbn or step_graph" --timeout 200 --timeout-method thread
step 600 ${TAG}_dist python3 -u -m pytest tests/test_gpu_dist.py -x -v -s --timeout 300 --timeout-method thread
step 300 ${TAG}_bench python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
grep -h "bwd reduce" gpurun_out/${TAG}_bnbase.log gpurun_out/${TAG}_bnnew.log
tail -2 gpurun_out/${TAG}_ktests.log gpurun_out/${TAG}_gen.log
grep -E "PASSED|FAILED|overlap:|FORCE" gpurun_out/${TAG}_dist.log | head
grep -h '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-300
