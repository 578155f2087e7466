#!/bin/bash
# decode parity (decode + stereo + multichannel), then the multiband / 2-band / batched legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/dec2
timeout -k 10 600 python -u -m pytest ${DEC_TESTS:-tests/test_gpu_decode.py tests/test_gpu_stereo.py tests/test_gpu_files.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/dec2/tests.log 2>&1 || { tail -60 gpurun_out/dec2/tests.log; exit 1; }
tail -2 gpurun_out/dec2/tests.log
timeout -k 10 300 python -u -c "
import json, sys
sys.path.insert(0, '.')
import bench
from flac_raster_amd import _native
ctx = _native.Context(0)
r = bench.convert_multiband(ctx)
print('multiband decode', json.dumps(r['decode']), flush=True)
ctx.close()
" > gpurun_out/dec2/legs.log 2>&1 || { tail -30 gpurun_out/dec2/legs.log; exit 1; }
cat gpurun_out/dec2/legs.log
