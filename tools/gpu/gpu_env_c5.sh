#!/bin/bash
# decode / C5 tests, then C5 latency with and without an env switch (ENVAB), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/envc5
timeout -k 10 600 python -u -m pytest ${C5_TESTS:-tests/test_gpu_decode.py tests/test_gpu_configs.py} -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/envc5/tests.log 2>&1 || { tail -60 gpurun_out/envc5/tests.log; exit 1; }
tail -2 gpurun_out/envc5/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu --steps 2 --queries 1000 > gpurun_out/envc5/a$rep.json 2> gpurun_out/envc5/a$rep.err || { tail -30 gpurun_out/envc5/a$rep.err; exit 1; }
  env $ENVAB timeout -k 10 300 python -u bench.py --no-extras --no-cpu --steps 2 --queries 1000 > gpurun_out/envc5/b$rep.json 2> gpurun_out/envc5/b$rep.err || { tail -30 gpurun_out/envc5/b$rep.err; exit 1; }
  python -c "
import json
for n in ('a','b'):
    d=json.load(open('gpurun_out/envc5/%s$rep.json'%n)); b=d['bbox_extract']; print(n, b['p50_ms'], b['p90_ms'], b['kernels_ms_rank0'])
"
done
