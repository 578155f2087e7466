#!/bin/bash
# Rehearsal of the driver's N = 2 bench on a one-GPU box: two ranks (torch.distributed.run) share the GPU and
# exchange tile sizes over the host (FRS_COMM_BACKEND=tcp; RCCL needs one GPU per rank).  -> gpurun_out/bench2/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_COMM_BACKEND=tcp
mkdir -p gpurun_out/bench2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29711 bench.py --gpus 2 --steps 5 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench2/bench.json 2> gpurun_out/bench2/bench.err || { tail -30 gpurun_out/bench2/bench.err; exit 1; }
cat gpurun_out/bench2/bench.json
