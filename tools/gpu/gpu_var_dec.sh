#!/bin/bash
# lane-decoder parity with the working-tree library, then batched-decode timing per prebuilt variant library
# (variants/lib<name>.so; "cur" = the working-tree build), alternating in one call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/vardec
FRS_LIB_PATH=${TESTLIB:-flac_raster_amd/libflac_raster_amd.so} timeout -k 10 600 python -u -m pytest ${DEC_TESTS:-tests/test_gpu_decode.py} -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/vardec/tests.log 2>&1 || { tail -60 gpurun_out/vardec/tests.log; exit 1; }
tail -2 gpurun_out/vardec/tests.log
for rep in 1 2; do
for v in ${VARIANTS:-cur}; do
  if [ "$v" = cur ]; then L=flac_raster_amd/libflac_raster_amd.so; else L=variants/lib$v.so; fi
  FRS_LIB_PATH=$L timeout -k 10 300 python -u tools/gpu/dec_bench.py 3 ${Q:-0} > gpurun_out/vardec/$v.$rep.json \
    2> gpurun_out/vardec/$v.$rep.err || { tail -30 gpurun_out/vardec/$v.$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/vardec/$v.$rep.json'))
print('$v', [ (b['ms'], b.get('kernels_ms')) for b in d['batched_decode']])
"
done
done
