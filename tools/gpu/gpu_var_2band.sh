#!/bin/bash
# convert_2band leg per prebuilt variant library (variants/lib<name>.so), alternating in one call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/var2b
for v in ${VARIANTS:-base}; do
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 300 python -u -c "
import json, sys
sys.path.insert(0, '.')
import bench
from flac_raster_amd import _native
ctx = _native.Context(0)
r = bench.convert_2band(ctx)
print('$v', r['ms_per_step'], r['kernels_ms'], flush=True)
ctx.close()
" > gpurun_out/var2b/$v.log 2>&1 || { tail -20 gpurun_out/var2b/$v.log; exit 1; }
  cat gpurun_out/var2b/$v.log
done
