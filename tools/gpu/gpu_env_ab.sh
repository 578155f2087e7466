#!/bin/bash
# Encode-parity tests, then the C4 step under alternating environment settings -> gpurun_out/envab/
# usage: AB="FRS_ANA_V4=0 FRS_ANA_V4=1" ./tools/gpu/gpu_env_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/envab/pytest.log 2>&1 || { tail -30 gpurun_out/envab/pytest.log; exit 1; }
tail -2 gpurun_out/envab/pytest.log
i=0
for kv in ${AB:-X=0}; do
  i=$((i+1))
  env $kv timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/envab/r$i.json 2> gpurun_out/envab/r$i.err || { tail -20 gpurun_out/envab/r$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/envab/r$i.json'));print('$kv', d['ms_per_step'], d['kernels_ms'])"
done
