#!/bin/bash
# Encode-parity tests, then the C4 step at FRS_ENC_SPLIT = 1..4 (same box) -> gpurun_out/split/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/split
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/split/pytest.log 2>&1 || { tail -30 gpurun_out/split/pytest.log; exit 1; }
tail -2 gpurun_out/split/pytest.log
for s in ${SPLITS:-1 2 3 4 1 2}; do
  FRS_ENC_SPLIT=$s timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/split/s$s.json 2> gpurun_out/split/s$s.err || { tail -20 gpurun_out/split/s$s.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/split/s$s.json'));print('split $s', d['ms_per_step'], d['kernels_ms'])"
done
