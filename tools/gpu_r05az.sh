#!/bin/bash
# grid size of the halo weight gradient (EEGAN_CONV wgrad_halo_blocks, default 512): in-process A/B
source ./run_gpu_steps.sh
TAG=${1:-r05az}
SH=d256_b0_3x3,c3x3_64_128,c3x3_32_256,c3x3_64_32_256
for b in 256 512 1024; do
  step 300 ${TAG}_cb$b env EEGAN_CONV=wgrad_halo_blocks=$b python3 tools/conv_bench.py --shapes $SH --dirs wgrad
done
for f in gpurun_out/${TAG}_cb*.log; do echo "== $f"; grep -E "TF/s" $f; done
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=wgrad_halo_blocks=256" "EEGAN_CONV=wgrad_halo_blocks=1024" --reps 4 --steps 20
tail -4 gpurun_out/${TAG}_ab.log
