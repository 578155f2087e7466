#!/bin/bash
# Round-4 first call: the N = 2 bench rehearsal test, then the base variant's parity + C4 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4/bench_test.log 2>&1 || { tail -30 gpurun_out/r4/bench_test.log; exit 1; }
tail -3 gpurun_out/r4/bench_test.log
VARIANTS="${VARIANTS:-base}" ./tools/gpu/gpu_var_ab.sh
