#!/bin/bash
# in-process A/B: real-image d_loss share of the small discriminators beside the generator's forward
source ./run_gpu_steps.sh
TAG=${1:-r05ak}
P=py:eegan_hip.trainer
step 900 ${TAG}_ab python3 -u tools/ab_inproc.py "$P.DREAL_EARLY=(1,)" "$P.DREAL_EARLY=(1,) $P.DREAL_LANE='damsm'" "$P.DREAL_EARLY=(0,1) $P.DREAL_LANE='damsm'" "$P.DREAL_EARLY=(2,) $P.DREAL_LANE='damsm'" --reps 3 --steps 20
tail -6 gpurun_out/${TAG}_ab.log
