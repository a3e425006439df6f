#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05l}
step 300 ${TAG}_head python3 tools/determinism.py --config C2 --reps 6 --steps 1
step 300 ${TAG}_nofuse env EEGAN_CONV=splitk_fused=0 python3 tools/determinism.py --config C2 --reps 6 --steps 1
for f in head nofuse; do echo "== $f"; grep -h "determinism\|G params" gpurun_out/${TAG}_$f.log | cut -c1-400; done
