#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
# kernel-trace + stats pass, then one PMC pass per counter (never combined
# with sys/runtime tracing).  Outputs under gpurun_out/prof_<tag>/.
TAG=${1:-r01}
STEPS=${2:-6}
CFG=${3:-C2}
source "$(dirname "$0")/../run_gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$TAG
mkdir -p $O
step 900 prof_trace rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --config $CFG --steps $STEPS --warmup 2 --no-cpu-baseline
step 900 prof_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
  python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --graph off --timing-steps 1 --op-log $O/ops.json
step 900 prof_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
  python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --graph off --timing-steps 1 --op-log $O/ops_x.json
step 900 prof_mfma rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- \
  python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --graph off --timing-steps 1 --op-log $O/ops_x.json
python3 tools/rocprof_families.py --trace $O/trace --fetch $O/fetch --write $O/write --mfma $O/mfma \
  --bench-line gpurun_out/prof_trace.log --ops $O/ops.json --config $CFG --out $O/families.json > /dev/null
python3 tools/dispatch_groups.py $O/trace --steps 0 --filter conv --top 60 > $O/conv_groups.txt
python3 -c "import json; d = json.load(open('$O/families.json')); [print('%-16s %6.1f MB/step excess  %5.2fx  %5.1f calls  %s' % (r['kind'], r['excess_MB_per_step'], r['pmc_over_algorithmic'] or 0, r['calls_per_step'], r['shape'])) for r in d.get('per_shape', [])[:40]]" > $O/per_shape_pmc.txt
python3 tools/dispatch_groups.py $O/trace --steps 0 --top 60 > $O/all_groups.txt
for d in trace fetch write mfma; do find $O/$d -name '*.csv' -size +20M -delete; done
ls -la $O
