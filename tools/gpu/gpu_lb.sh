#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_lb.log 2>&1 || exit 1
FRS_ABLATE=64 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/lb.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/lb0.log 2>&1
