#!/bin/bash
# Standard GPU cycle on the box: kernel + model parity tests, per-shape
# profile, bench line.  Stops at the first crash/timeout (run_gpu_steps.sh).
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 600 kernels python3 -m pytest tests/test_gpu_kernels.py -x -q
step 900 models python3 -m pytest tests/test_gpu_models.py -q -s
step 600 shapes python3 tools/profile_step.py --steps 2 --out gpurun_out/shapes.json
step 600 bench python3 bench.py --no-cpu-baseline
grep -h '"metric"' gpurun_out/bench.log
