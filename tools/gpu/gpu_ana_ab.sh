#!/bin/bash
# Analysis A/B: parity (encode + files) with the role-split analysis (FRS_ANA_V5=1), then the C4 step with each form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ana
FRS_ANA_V5=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_files.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ana/v5.pytest.log 2>&1 || { echo "v5 parity FAILED"; tail -30 gpurun_out/ana/v5.pytest.log; exit 1; }
tail -2 gpurun_out/ana/v5.pytest.log
for v in ${ANA_FORMS:-0 1 0 1}; do
  FRS_ANA_V5=$v timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/ana/b$v.json 2> gpurun_out/ana/b$v.err || { tail -20 gpurun_out/ana/b$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ana/b$v.json'));print('v5=$v', d['ms_per_step'], d['kernels_ms'])"
done
