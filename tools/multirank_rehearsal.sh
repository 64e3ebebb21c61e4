#!/bin/bash
# Two ranks on one GPU (gloo reductions): rehearses the multi-rank bench path and its memory footprint.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mr
BCP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/mr/bench2.log 2>&1
tail -n 1 gpurun_out/mr/bench2.log
