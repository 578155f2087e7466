#!/bin/bash
# Default bench line (N = 1, all extras) -> gpurun_out/bench/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/bench
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench.err || { tail -30 gpurun_out/bench/bench.err; exit 1; }
cat gpurun_out/bench/bench.json
