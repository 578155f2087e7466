#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: 2 ranks share the GPU, gloo carries the all-gather
# (RCCL refuses two ranks on one device).  Small raster to keep it short.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --height 8192 --width 8192 --backend gloo --queries 50 --no-cpu > gpurun_out/mgpu.log 2>&1
echo "rc=$?" >> gpurun_out/mgpu.log
