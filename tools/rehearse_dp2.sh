#!/bin/bash
# Rehearse the N=2 data-parallel bench path on a ONE-GPU box: two ranks share
# cuda:0 and talk over gloo (RCCL refuses two ranks on one device).  Checks the
# multi-rank code path (SyncBN all-reduce, DAMSM gathers, gradient averaging,
# max-over-ranks timing), not multi-GPU performance.
cd "${GRAFT_REPO_ROOT:-.}"
EEGAN_SHARE_GPU=1 EEGAN_DIST_BACKEND=gloo EEGAN_GRAPH_DIST=0 timeout -k 10 600 \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --timing-steps 1
