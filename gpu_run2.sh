#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python dbg_decode.py > gpurun_out/dbg_decode.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_prof.log 2>&1
echo "done rc=$?"
