#!/bin/bash
# round 4 development cycle: device-visibility probe, all -m gpu tests (parity log), bench line
source ./run_gpu_steps.sh
TAG=${1:-r04a}
export EEGAN_PARITY_LOG=$PWD/gpurun_out/${TAG}_parity_log.txt
rm -f "$EEGAN_PARITY_LOG"
step 120 ${TAG}_probe python3 -c "
import os, torch
print({k: os.environ.get(k) for k in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES')})
print('device_count before init', torch.cuda.device_count(), 'initialized', torch.cuda.is_initialized())
print('after init', torch.cuda.device_count(), torch.cuda.get_device_name(0))
"
step 1000 ${TAG}_gputests python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step 400 ${TAG}_bench python3 bench.py --cpu-seconds 5
grep -h '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-400
