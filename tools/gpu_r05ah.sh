#!/bin/bash
# GP mask detach scoped to the trainer: tests (models, dist), in-process A/B
source ./run_gpu_steps.sh
TAG=${1:-r05ah}
step 900 ${TAG}_tests python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "gradient_penalty or full_step or graph_matches_eager or deterministic or real_early"
step 900 ${TAG}_dist python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=" "py:eegan_hip.functional.GP_DETACH_MASKS=False" --reps 3 --steps 20
tail -4 gpurun_out/${TAG}_ab.log
