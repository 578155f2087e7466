#!/bin/bash
# two-channel fast path: stereo + multi-band parity, then the convert_2band / convert_multiband legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/stereo
timeout -k 10 600 python -u -m pytest ${ST_TESTS:-tests/test_gpu_stereo.py tests/test_gpu_levels.py tests/test_gpu_files.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/stereo/tests.log 2>&1 || { tail -60 gpurun_out/stereo/tests.log; exit 1; }
tail -2 gpurun_out/stereo/tests.log
timeout -k 10 300 python -u -c "
import json, sys
sys.path.insert(0, '.')
import bench
from flac_raster_amd import _native
ctx = _native.Context(0)
for leg in (bench.convert_2band, bench.convert_multiband):
    print(leg.__name__, json.dumps(leg(ctx)), flush=True)
ctx.close()
" > gpurun_out/stereo/legs.log 2>&1 || { tail -30 gpurun_out/stereo/legs.log; exit 1; }
cat gpurun_out/stereo/legs.log
