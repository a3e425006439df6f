#!/bin/bash
# GP second backward without the zero-gradient forward-graph passes: trace, tests, A/B
source ./run_gpu_steps.sh
TAG=${1:-r05ag}
step 240 ${TAG}_gptrace python3 tools/gp_trace.py
grep -v amdgpu gpurun_out/${TAG}_gptrace.log | head -20
step 900 ${TAG}_tests python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "gradient_penalty or full_step or graph_matches_eager or deterministic or real_early"
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=" "py:eegan_hip.functional.DETACH_MASK_SRC=False" --reps 3 --steps 20
tail -4 gpurun_out/${TAG}_ab.log
