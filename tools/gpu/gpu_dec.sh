#!/bin/bash
# C5 decode A/B: default (scalar-unit frame decoder) vs FRS_ABLATE=1024 (lane-0 decoder), 200 queries each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/dec; mkdir -p gpurun_out/dec
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --queries 200 > gpurun_out/dec/scalar.log 2>&1 || exit 1
FRS_ABLATE=1024 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --queries 200 > gpurun_out/dec/lane0.log 2>&1 || exit 1
echo done
