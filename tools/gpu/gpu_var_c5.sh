#!/bin/bash
# C5 latency per variant library (variants/lib<name>.so; "cur" = the working-tree build), alternating, after the
# decode / C5 tests with the working-tree library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/varc5
if [ -n "${C5_TESTS:-tests/test_gpu_decode.py tests/test_gpu_configs.py}" ]; then
  timeout -k 10 600 python -u -m pytest ${C5_TESTS:-tests/test_gpu_decode.py tests/test_gpu_configs.py} -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/varc5/tests.log 2>&1 || { tail -60 gpurun_out/varc5/tests.log; exit 1; }
  tail -2 gpurun_out/varc5/tests.log
fi
for rep in 1 2; do
for v in ${VARIANTS:-cur}; do
  if [ "$v" = cur ]; then L=flac_raster_amd/libflac_raster_amd.so; else L=variants/lib$v.so; fi
  FRS_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-extras --no-cpu --steps 2 --queries ${Q:-1000} \
    > gpurun_out/varc5/$v.$rep.json 2> gpurun_out/varc5/$v.$rep.err || { tail -30 gpurun_out/varc5/$v.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/varc5/$v.$rep.json'));b=d['bbox_extract'];print('$v',b['p50_ms'],b['p90_ms'],b['kernels_ms_rank0'])"
done
done
