#!/bin/bash
# decode parity tests, then dec_bench per decode variant (variants/lib<name>.so), then FETCH/WRITE PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dec
timeout -k 10 400 python -u -m pytest ${DEC_TESTS:-tests/test_gpu_decode.py tests/test_gpu_stereo.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/dec/tests.log 2>&1 || { tail -40 gpurun_out/dec/tests.log; exit 1; }
tail -1 gpurun_out/dec/tests.log
for v in ${VARIANTS:-}; do
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 200 python -u tools/gpu/dec_bench.py 2 200 > gpurun_out/dec/$v.json 2> gpurun_out/dec/$v.err || { tail -20 gpurun_out/dec/$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/dec/$v.json'));b=d['batched_decode'][-1];q=d['bbox_extract'];print('$v',b['ms'],b['kernels_ms'],q['p50_ms'],q['p90_ms'])"
done
[ -n "$NOPMC" ] && exit 0
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/gpurun_out/dec/pmc_$c -o pmc -- python3 $GRAFT_REPO_ROOT/tools/gpu/dec_bench.py 1 0 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/dec/pmc_$c.err || exit 1
done
echo pmc done
