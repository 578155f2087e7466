#!/bin/bash
# timeline of C5 queries: kernel + memory-copy trace (no counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/c5trace
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c5trace/raw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-cpu --steps 1 --warmup 1 --queries 60 > $GRAFT_REPO_ROOT/gpurun_out/c5trace/b.json 2> $GRAFT_REPO_ROOT/gpurun_out/c5trace/b.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c5trace/b.err; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/c5trace/raw -name "*.csv" | head
