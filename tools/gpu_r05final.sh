#!/bin/bash
# round-5 evidence: device probe + all -m gpu tests (parity log) + bench line, then phases + rocprof trace / PMC
TAG=${1:-r05c}
bash tools/gpu_r04a.sh $TAG || exit $?
bash tools/gpu_r05w2.sh $TAG
