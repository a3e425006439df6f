#!/bin/bash
# BN kernels: kernel + model tests, then library A/B on the replayed step
source ./run_gpu_steps.sh
TAG=${1:-bn}
step 300 ${TAG}_tests python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "bn or BN or generator or syncbn" --timeout 120 --timeout-method thread
ROUNDS=${ROUNDS:-2} bash tools/gpu_lib_ab.sh
