#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05ar}
SH=c3x3_32_256,c3x3_32_128,c3x3_64_32_256,c3x3_64_32_128,img_32_256
step 300 ${TAG}_cb_def python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd
step 300 ${TAG}_cb_nothin env EEGAN_CONV=thin=0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd
step 300 ${TAG}_cb_nothinlds env EEGAN_CONV=thin_lds=0 python3 tools/conv_bench.py --shapes $SH --dirs fwd,bwdd
for f in gpurun_out/${TAG}_cb_*.log; do echo "== $f"; grep -E "TF/s" $f; done
