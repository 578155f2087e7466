#!/bin/bash
# decode parity, then the batched decode + multiband legs (both span checks)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/dec
timeout -k 10 600 python -u -m pytest ${DEC_TESTS:-tests/test_gpu_decode.py tests/test_gpu_stereo.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/dec/tests.log 2>&1 || { tail -60 gpurun_out/dec/tests.log; exit 1; }
tail -2 gpurun_out/dec/tests.log
for sr in 0 1; do
FRS_SPAN_READ=$sr timeout -k 10 300 python -u bench.py --no-cpu --queries 0 --steps 3 > gpurun_out/dec/b$sr.json 2> gpurun_out/dec/b$sr.err || { tail -30 gpurun_out/dec/b$sr.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/dec/b$sr.json'))
print('span_read=$sr', 'batched', json.dumps(d['batched_decode']))
print('  multiband', json.dumps(d['convert_multiband']['decode']))
"
done
