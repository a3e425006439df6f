#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05ao}
step 400 ${TAG}_tests python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad"
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=wgrad_halo=0" --reps 4 --steps 20
tail -3 gpurun_out/${TAG}_ab.log
