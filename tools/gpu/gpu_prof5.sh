#!/bin/bash
# Round profile (v7): GPU parity tests, kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes, default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof5
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/prof5/pytest.log 2>&1 || exit 1
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --queries 200"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5/kt -o run -- $B > gpurun_out/prof5/kt.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof5/fetch -o run -- $B > gpurun_out/prof5/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof5/write -o run -- $B > gpurun_out/prof5/write.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/prof5/bench_default.log 2>&1 || exit 1
echo done
