#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu4.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu4.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-tiles 79 > gpurun_out/bench4.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench4.log
