#!/bin/bash
# PMC HBM traffic of the 64-channel 3x3 kernels: conv_halo3r vs conv_halo3 (conv_bench, D256 b0 shape)
source ./run_gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_halo
mkdir -p $O
for v in 1 0; do
  step 120 pmc_fetch_$v env EEGAN_CONV=halo_r=$v timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- python3 tools/conv_bench.py --shapes d256_b0_3x3 --dirs fwd,bwdd --iters 5
  step 120 pmc_write_$v env EEGAN_CONV=halo_r=$v timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$v -o run -- python3 tools/conv_bench.py --shapes d256_b0_3x3 --dirs fwd,bwdd --iters 5
done
python3 - <<'PY'
import csv, glob, collections
for v in ('1', '0'):
    for cnt in ('fetch', 'write'):
        agg = collections.defaultdict(lambda: [0.0, 0])
        for f in glob.glob('gpurun_out/pmc_halo/%s_%s/**/*counter_collection.csv' % (cnt, v), recursive=True):
            for r in csv.DictReader(open(f)):
                n = r['Kernel_Name']
                if 'halo3' not in n:
                    continue
                k = n.split('(')[0].replace('void ', '')[:60]
                agg[k][0] += float(r['Counter_Value']); agg[k][1] += 1
        for k, (s, c) in agg.items():
            print('halo_r=%s %-6s %-60s %10.1f KB per dispatch (%d)' % (v, cnt, k, s / max(c, 1), c))
PY
