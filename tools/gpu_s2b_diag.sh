#!/bin/bash
# stride-2 halo backward-data: bit-identity tests, grid size and phase knock-outs
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 300 ktest python3 -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "s2bwd or fast_path"
for B in 512 1024 2048; do
  step 100 s2b_b$B env EEGAN_CONV_S2B_BLOCKS=$B python3 tools/conv_bench.py --shapes c4x4s2_32_256 --dirs bwdd --device-time
done
step 100 s2b_nl2 env EEGAN_CONV_NOLOAD=2 python3 tools/conv_bench.py --shapes c4x4s2_32_256 --dirs bwdd --device-time
for f in gpurun_out/s2b_*.log; do echo "$f: $(grep bwdd $f)"; done
