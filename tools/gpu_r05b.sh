#!/bin/bash
# round 5: the data-parallel drop-in (rank shards, broadcast), peer fast-poison, branched generator bit-identity,
# the tightened gates
source ./run_gpu_steps.sh
TAG=${1:-r05b}
export EEGAN_PARITY_LOG=$PWD/gpurun_out/${TAG}_parity_log.txt
rm -f "$EEGAN_PARITY_LOG"
step 600 ${TAG}_tests python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_peer.py tests/test_gpu_pipeline.py "tests/test_gpu_models.py::test_generator" "tests/test_gpu_models.py::test_generator_branched_matches_single_stream" -x -v -s --timeout 300 --timeout-method thread
grep -E "PASS|FAIL|DP2|PARITY gen" gpurun_out/${TAG}_tests.log | head -60
