#!/bin/bash
# Planner-knob sweep on the small-spatial conv shapes (device time per call).
cd "$GRAFT_REPO_ROOT"
S=c3x3_768_4,c3x3_512_4,c4x4s4_1024_4,c3x3_256_8,c4x4s2_512_8,c3x3_512_8,c1x1_768_17,c1x1_32_256,c3x3_512_16
for cfg in "512 16" "1024 8" "2048 4" "1024 16" "2048 8"; do
  set -- $cfg
  echo "=== TARGET=$1 MINK=$2"
  EEGAN_CONV_TARGET=$1 EEGAN_CONV_MINK=$2 timeout -k 10 120 python3 tools/conv_bench.py --device-time --iters 20 --shapes $S || exit 1
done
