#!/bin/bash
# PMC counters of one kernel (KF, default conv_halo3_kernel) under CMD (default: conv_bench on
# one shape), one pass per counter group (diagnostic)
source ./run_gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-hp}
SH=${SH:-c3x3_128_64}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  step 120 ${TAG}_p$i timeout -s KILL 100 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_p$i -o run -- \
    ${CMD:-python3 tools/conv_bench.py --shapes $SH --dirs fwd --iters 5}
done
python3 - "$TAG" "${KF:-halo3}" <<'PY'
import csv, glob, sys, collections
tag, kf = sys.argv[1], sys.argv[2]
for i in (1, 2):
    acc = collections.defaultdict(list)
    for f in glob.glob('gpurun_out/%s_p%d/**/*counter_collection.csv' % (tag, i), recursive=True):
        for r in csv.DictReader(open(f)):
            if kf in r['Kernel_Name']:
                acc[(r['Dispatch_Id'], r['Counter_Name'])].append(float(r['Counter_Value']))
    per = collections.defaultdict(list)
    for (d, c), v in acc.items():
        per[c].append(sum(v))
    for c, v in sorted(per.items()):
        print('pass%d %-28s mean %.4g over %d dispatches' % (i, c, sum(v) / len(v), len(v)))
PY
find gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 -name '*.csv' -size +5M -delete
