#!/bin/bash
# Deep-ring sweep on the small-grid conv shapes (device time per call), then
# bench A/B (4-stage rings everywhere vs the deep ring on small grids).
cd "$GRAFT_REPO_ROOT"
S=c3x3_768_4,c3x3_512_4,c4x4s4_1024_4,c3x3_256_8,c4x4s2_512_8,c3x3_512_8,c1x1_768_17,c3x3_512_16,c3x3_256_32,c3x3_128_64
for st in 4 6 8; do
  echo "=== DEEP_STAGES=$st"
  EEGAN_CONV_DEEP_STAGES=$st timeout -k 10 120 python3 tools/conv_bench.py --device-time --iters 20 --shapes $S --dirs fwd,bwdd || exit 1
done
for st in 4 8 4 8; do
  echo "=== bench DEEP_STAGES=$st"
  EEGAN_CONV_DEEP_STAGES=$st timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-timer --steps 20 | grep -o '"value": [0-9.]*' || exit 1
done
