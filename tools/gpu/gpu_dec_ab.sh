#!/bin/bash
# Decoder A/B: per variant library, the decode parity tests then dec_bench (batched decode of the C4 arena + C5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dec
for v in ${VARIANTS:-dbase}; do
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stereo.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/dec/$v.tests.log 2>&1 || { echo "$v: decode tests FAILED"; tail -30 gpurun_out/dec/$v.tests.log; exit 1; }
  tail -1 gpurun_out/dec/$v.tests.log
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 200 python -u tools/gpu/dec_bench.py 3 200 > gpurun_out/dec/$v.json 2> gpurun_out/dec/$v.err || { tail -20 gpurun_out/dec/$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/dec/$v.json'));b=d['batched_decode'];q=d['bbox_extract'];print('$v',[x['ms'] for x in b],b[-1]['kernels_ms'],q['p50_ms'],q['p90_ms'])"
done
