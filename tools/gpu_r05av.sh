#!/bin/bash
# in-launch dot finish: kernel + model tests, in-process A/B
source ./run_gpu_steps.sh
TAG=${1:-r05av}
step 600 ${TAG}_tests python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_models.py -k "dot or gradient_penalty or scale or full_step or graph_matches_eager or deterministic or discriminator"
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "py:eegan_hip.functional.DOT_FINISH_FUSED=False" --reps 4 --steps 20
tail -3 gpurun_out/${TAG}_ab.log
