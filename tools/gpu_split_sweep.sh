# conv_bench of the small-grid split-K shapes under environment variants
# (planner knobs / diagnostics), kernel + split-K reduce times per launch
set -o pipefail
mkdir -p gpurun_out
S=${SHAPES:-c3x3_512_4,c3x3_768_4,c3x3_256_8,c3x3_512_8,c4x4s2_512_8}
IFS=';' read -ra CFGS <<< "${CFGS:-;EEGAN_CONV_KS=2;EEGAN_CONV_KS=2 EEGAN_CONV_NOLOAD=1;EEGAN_CONV_NOLOAD=4;EEGAN_CONV_KS=2 EEGAN_CONV_NOLOAD=5}"
for cfg in "${CFGS[@]}"; do
  echo "=== cfg: $cfg"
  env $cfg timeout -k 10 120 python tools/conv_bench.py --shapes $S --dirs ${DIRS:-fwd} --iters 50 --device-time || exit 1
done
