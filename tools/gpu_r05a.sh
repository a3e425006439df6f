#!/bin/bash
# Round-5 baseline on this box: D256 conv shapes (all directions) + the C2 bench line.
source ./run_gpu_steps.sh
TAG=${1:-r05a}
S=${S:-d256_b0_s2,d256_b0_3x3,d256_b1_s2,d256_b1_3x3,d256_b2_s2,d256_b2_3x3,d256_b3_s2,d256_b3_3x3,d256_b4_s2,d256_b4_3x3,d256_b5_s2,d256_b5_3x3,c3x3_512_4,c3x3_256_8,c3x3_512_8,c4x4s2_512_8}
step 300 ${TAG}_cb python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd,wgrad --device-time
step 300 ${TAG}_bench python3 bench.py --steps 20 --warmup 5
