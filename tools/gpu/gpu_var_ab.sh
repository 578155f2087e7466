#!/bin/bash
# Per variant library (variants/lib<name>.so): encode-parity tests, then the C4 step (20 timed steps) -> gpurun_out/var/
# usage: VARIANTS="base ilp" ./tools/gpu/gpu_var_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/var
for v in ${VARIANTS:-base}; do
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/var/$v.pytest.log 2>&1 || { echo "$v: parity FAILED"; tail -15 gpurun_out/var/$v.pytest.log; exit 1; }
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err || { tail -20 gpurun_out/var/$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/var/$v.json'));print('$v', d['ms_per_step'], d['kernels_ms'])"
done
