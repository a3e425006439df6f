#!/bin/bash
# CPU-baseline binding A/B on the GPU box (OMP_PROC_BIND close / false / spread, 16 threads),
# then an in-process A/B of the SyncBN grid knobs (profiles/r06n_cpu_binding_ab.txt, r06n_bn_grid_ab.txt)
source ./run_gpu_steps.sh
A=$(nproc)
for v in "close cores" "false none" "spread cores"; do
  set -- $v
  if [ "$2" = none ]; then
    step 200 cpuab_$1 env EEGAN_CPU_AFFINITY=$A EEGAN_CPU_SHARE=16 OMP_NUM_THREADS=16 OMP_PROC_BIND=$1 python3 bench.py --cpu-baseline-only --cpu-seconds 15 || exit $?
  else
    step 200 cpuab_$1 env EEGAN_CPU_AFFINITY=$A EEGAN_CPU_SHARE=16 OMP_NUM_THREADS=16 OMP_PROC_BIND=$1 OMP_PLACES=$2 python3 bench.py --cpu-baseline-only --cpu-seconds 15 || exit $?
  fi
  grep -h '"value"' gpurun_out/cpuab_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['value'],3), d['timed_spread'], d['timed_iqr_spread'], d['sample'][-60:])"
done
step 900 bnk_ab python3 -u tools/ab_inproc.py "EEGAN_BN=bwd_target=2048" "EEGAN_BN=bwd_target=512" "EEGAN_BN=dx_target=1024" "EEGAN_BN=fwd_target=3072" "EEGAN_CONV=mink=24" --reps 3 --steps 30
