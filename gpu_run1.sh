#!/bin/bash
# first GPU pass: build check, parity tests, smoke, small bench, rocprof of the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocminfo | grep -m2 gfx > gpurun_out/rocminfo.txt 2>&1
timeout -k 10 300 python -m pytest tests/test_gpu_encode_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --height 16384 --width 16384 --steps 3 --warmup 1 --cpu-tiles 64 > gpurun_out/bench_c3.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1
echo "done rc=$?"
