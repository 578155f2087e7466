#!/bin/bash
# decode tests, then the batched decode with and without an env switch (ENVAB, e.g. FRS_SPAN_B8=1), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/envdec
timeout -k 10 600 python -u -m pytest ${DEC_TESTS:-tests/test_gpu_decode.py tests/test_gpu_configs.py} -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/envdec/tests.log 2>&1 || { tail -60 gpurun_out/envdec/tests.log; exit 1; }
tail -2 gpurun_out/envdec/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u tools/gpu/dec_bench.py 3 0 > gpurun_out/envdec/a$rep.json 2> gpurun_out/envdec/a$rep.err || { tail -30 gpurun_out/envdec/a$rep.err; exit 1; }
  env $ENVAB timeout -k 10 300 python -u tools/gpu/dec_bench.py 3 0 > gpurun_out/envdec/b$rep.json 2> gpurun_out/envdec/b$rep.err || { tail -30 gpurun_out/envdec/b$rep.err; exit 1; }
  python -c "
import json
for n in ('a','b'):
    d=json.load(open('gpurun_out/envdec/%s$rep.json'%n)); print(n, [(b['ms'], b['kernels_ms']) for b in d['batched_decode']])
"
done
