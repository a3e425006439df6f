#!/bin/bash
# determinism A/B: round-4 snapshot (_r4) vs head, multi-stream C2 eager steps
source ./run_gpu_steps.sh
TAG=${1:-r05h}
step 300 ${TAG}_r4 bash -c "cd _r4 && python3 tools/determinism.py --config C2 --reps 5 --steps 2"
step 300 ${TAG}_head_noside python3 -c "
import sys; sys.argv=['x','--config','C2','--reps','5','--steps','2']
sys.path[:0]=['ee-gan_amd','.']
import eegan_hip.trainer as TR; TR.GEN_SIDE=False
import runpy; runpy.run_path('tools/determinism.py', run_name='__main__')"
grep -h "determinism" gpurun_out/${TAG}_*.log
