#!/bin/bash
# Input pipeline on the GPU box: parity tests and throughput.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 300 pipetests python3 -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread
step 300 pipebench python3 -u tools/pipeline_bench.py --batch 16
step 300 pipebench32 python3 -u tools/pipeline_bench.py --batch 32
grep -h '"batch"' gpurun_out/pipebench*.log
