#!/bin/bash
# Round profile: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE passes (separate runs), then a default
# bench line (with the CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
B="python3 bench.py --steps 5 --warmup 2 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2/kt -o run -- $B > gpurun_out/prof2/kt.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof2/fetch -o run -- $B > gpurun_out/prof2/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof2/write -o run -- $B > gpurun_out/prof2/write.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/prof2/bench_default.log 2>&1 || exit 1
echo done
