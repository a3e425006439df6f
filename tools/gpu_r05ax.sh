#!/bin/bash
# PMC HBM traffic of the 3x3 weight gradients: conv_wgrad_halo3 vs the tile path (D256 b0 and 32-ch 256^2 shapes)
source ./run_gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_wg
mkdir -p $O
for v in 1 0; do
  for sh in d256_b0_3x3 c3x3_32_256; do
    step 120 pmcw_f_${v}_$sh env EEGAN_CONV=wgrad_halo=$v timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_${v}_$sh -o run -- python3 tools/conv_bench.py --shapes $sh --dirs wgrad --iters 5
    step 120 pmcw_w_${v}_$sh env EEGAN_CONV=wgrad_halo=$v timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_${v}_$sh -o run -- python3 tools/conv_bench.py --shapes $sh --dirs wgrad --iters 5
  done
done
python3 - <<'PY'
import csv, glob, collections, re
for v in ('1', '0'):
    for sh in ('d256_b0_3x3', 'c3x3_32_256'):
        tot = {}
        for cnt in ('fetch', 'write'):
            agg = collections.defaultdict(lambda: [0.0, 0])
            for f in glob.glob('gpurun_out/pmc_wg/%s_%s_%s/**/*counter_collection.csv' % (cnt, v, sh), recursive=True):
                for r in csv.DictReader(open(f)):
                    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '')
                    if 'wgrad' not in n and 'colsum' not in n and 'reduce' not in n:
                        continue
                    k = re.sub(r'\(.*$', '', n)[:50]
                    agg[k][0] += float(r['Counter_Value']); agg[k][1] += 1
            for k, (s, c) in agg.items():
                print('wgrad_halo=%s %-12s %-6s %-50s %10.1f KB per dispatch (%d)' % (v, sh, cnt, k, s / max(c, 1), c))
PY
