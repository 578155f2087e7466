#!/bin/bash
# Round-4 A/B batch: role-split analysis parity + step, encoder variants, lane-decoder variants, 3-wave C5 decoder
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dec
./tools/gpu/gpu_ana_ab.sh || exit 1
VARIANTS="${ENC_VARIANTS:-base crc2 pwt2 early early_crc2}" ./tools/gpu/gpu_var_ab.sh || exit 1
# C5 decoder: resolver + builders (FRS_PIPE2=1) parity, then C5 latency with each form
FRS_PIPE2=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py -k "pipe2 or c5_bbox" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/dec/pipe2.tests.log 2>&1 || { echo "pipe2 tests FAILED"; tail -30 gpurun_out/dec/pipe2.tests.log; exit 1; }
tail -1 gpurun_out/dec/pipe2.tests.log
for v in 0 1; do
  FRS_PIPE2=$v timeout -k 10 200 python -u tools/gpu/dec_bench.py 1 300 > gpurun_out/dec/pipe2_$v.json 2> gpurun_out/dec/pipe2_$v.err || { tail -20 gpurun_out/dec/pipe2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/dec/pipe2_$v.json'));q=d['bbox_extract'];print('pipe2=$v',q['p50_ms'],q['p90_ms'],q['kernels_ms_rank0'])"
done
VARIANTS="${DEC_VARIANTS:-dbase dlean}" ./tools/gpu/gpu_dec_ab.sh || exit 1
