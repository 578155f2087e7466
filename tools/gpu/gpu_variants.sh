#!/bin/bash
# Bench line per prebuilt variant library (variants/lib<name>.so, tools/enc_ablate.py) -> gpurun_out/var/<name>.json
# usage: VARIANTS="base nocrc" BENCH_ARGS="..." ./tools/gpu/gpu_variants.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/var
for v in ${VARIANTS:-base}; do
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-extras --no-cpu --queries 0 --steps 10} \
    > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err || { tail -30 gpurun_out/var/$v.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/var/$v.json'));print('$v',d['ms_per_step'],d['kernels_ms'])"
done
