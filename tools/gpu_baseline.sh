#!/bin/bash
# Fresh-box baseline: every -m gpu test (parity log kept), the default bench
# line, the profiler's counter list and one MFMA-busy PMC pass over an eager
# step (each counter pass in its own run).
source "$(dirname "$0")/../run_gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-base}
export EEGAN_PARITY_LOG=gpurun_out/parity_$TAG.txt
rm -f "$EEGAN_PARITY_LOG"
step 900 gputests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s
step 600 bench python3 bench.py --no-cpu-baseline
grep -h '"metric"' gpurun_out/bench.log
step 120 counters rocprofv3 -L
step 300 pmc_mfma rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --graph off --no-timer
ls -R gpurun_out/pmc_mfma | head -20
