#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu16.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu16.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench16.log 2>&1 || exit 1
echo done
