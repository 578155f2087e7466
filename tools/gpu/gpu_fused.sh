#!/bin/bash
# k_fused_v6 (analysis + encode in one launch, FRS_FUSED=1): parity (encode, C3/C4 configs, files), then the C4 step
# against the two-launch form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fused
FRS_FUSED=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_encode_parity.py tests/test_gpu_configs.py tests/test_gpu_files.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/fused/parity.log 2>&1 || { echo "fused parity FAILED"; tail -30 gpurun_out/fused/parity.log; exit 1; }
tail -1 gpurun_out/fused/parity.log
for v in ${FORMS:-0 1 0 1}; do
  FRS_FUSED=$v timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/fused/b$v.json 2> gpurun_out/fused/b$v.err || { tail -20 gpurun_out/fused/b$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fused/b$v.json'));print('fused=$v', d['ms_per_step'], d['kernels_ms'])"
done
