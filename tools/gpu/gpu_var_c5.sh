#!/bin/bash
# C5 latency per prebuilt variant library (variants/lib<name>.so), alternating in one call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/varc5
for v in ${VARIANTS:-base}; do
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 300 python -u bench.py --no-extras --no-cpu --steps 2 --queries ${Q:-1000} \
    > gpurun_out/varc5/$v.json 2> gpurun_out/varc5/$v.err || { tail -30 gpurun_out/varc5/$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/varc5/$v.json'));b=d['bbox_extract'];print('$v',b['p50_ms'],b['p90_ms'],b['kernels_ms_rank0'])"
done
