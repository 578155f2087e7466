#!/bin/bash
# Round profile (v8): GPU parity tests, kernel-trace stats, FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes,
# default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/prof6; mkdir -p gpurun_out/prof6
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/prof6/pytest.log 2>&1 || exit 1
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --queries 200"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/kt -o run -- $B > gpurun_out/prof6/kt.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof6/fetch -o run -- $B > gpurun_out/prof6/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof6/write -o run -- $B > gpurun_out/prof6/write.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/prof6/valu -o run -- $B > gpurun_out/prof6/valu.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/prof6/bench_default.log 2>&1 || exit 1
echo done
