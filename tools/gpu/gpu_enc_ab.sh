#!/bin/bash
# encoder parity tests with the working-tree library, then the C4 step per variant library, alternating twice
# (variants/lib<name>.so; "cur" = the working-tree build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/encab
timeout -k 10 900 python -u -m pytest ${ENC_TESTS:-tests/test_gpu_encode_parity.py tests/test_gpu_configs.py tests/test_gpu_stereo.py tests/test_gpu_files.py} \
  -x -v --timeout 300 --timeout-method thread > gpurun_out/encab/tests.log 2>&1 || { tail -60 gpurun_out/encab/tests.log; exit 1; }
tail -2 gpurun_out/encab/tests.log
for rep in 1 2; do
for v in ${VARIANTS:-base cur}; do
  if [ "$v" = cur ]; then L=flac_raster_amd/libflac_raster_amd.so; else L=variants/lib$v.so; fi
  FRS_LIB_PATH=$L timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-extras --no-cpu --queries 0 --steps 10} \
    > gpurun_out/encab/$v.$rep.json 2> gpurun_out/encab/$v.$rep.err || { tail -30 gpurun_out/encab/$v.$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/encab/$v.$rep.json'));print('$v',d['ms_per_step'],d['kernels_ms'])"
done
done
