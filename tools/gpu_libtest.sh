#!/bin/bash
# kernel tests of the in-tree library, then library A/B (tools/ab_lib/libeegan_hip_base.so vs in-tree)
source ./run_gpu_steps.sh
TAG=${1:-lt}
step 300 ${TAG}_ktests python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread
ROUNDS=${ROUNDS:-3} bash tools/gpu_lib_ab.sh
