#!/bin/bash
# C5 path: pipe-decoder parity, then the C4 step + 1000 bbox queries (twice)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest ${C5_TESTS:-tests/test_gpu_decode.py tests/test_gpu_configs.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/c5/tests.log 2>&1 || { tail -60 gpurun_out/c5/tests.log; exit 1; }
tail -2 gpurun_out/c5/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-extras --no-cpu --steps 5 --queries 1000 > gpurun_out/c5/b$r.json 2> gpurun_out/c5/b$r.err || { tail -30 gpurun_out/c5/b$r.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/c5/b$r.json')); b=d['bbox_extract']
print('step', d['ms_per_step'], 'p50', b['p50_ms'], 'p90', b['p90_ms'], b['kernels_ms_rank0'])"
done
