#!/bin/bash
# encode parity files (product default), then C4-step bench lines alternating environment settings
# usage: ENVS="FRS_ENC_V=3 FRS_ENC_V=4 ..." [AB_TESTS=...] [AB_NOTESTS=1] ./tools/gpu/gpu_env_ab2.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/envab
if [ -z "$AB_NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests/test_gpu_encode_parity.py tests/test_gpu_configs.py tests/test_gpu_files.py tests/test_gpu_stride.py tests/test_gpu_stereo.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/envab/tests.log 2>&1 || { tail -60 gpurun_out/envab/tests.log; exit 1; }
tail -2 gpurun_out/envab/tests.log
fi
i=0
for e in ${ENVS:-FRS_ENC_V=3 FRS_ENC_V=4}; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-extras --no-cpu --queries 0 --steps 20} \
    > gpurun_out/envab/$i.json 2> gpurun_out/envab/$i.err || { tail -30 gpurun_out/envab/$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/envab/$i.json'));print('$e',d['ms_per_step'],d['kernels_ms'],d['config']['compressed_bytes_total'])"
done
