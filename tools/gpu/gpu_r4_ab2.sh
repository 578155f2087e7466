#!/bin/bash
# Round 4: role-split analysis ratios (FRS_ANA_V5=1: 4+4 waves, 2: 6+2) with wave-cycle counters, parity of both,
# the C4 step A/B, then the level 0..8 / loose mid/side GPU byte tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ana2
for v in 1 2; do
  FRS_ANA_V5=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ana2/v$v.pytest.log 2>&1 || { echo "v5=$v parity FAILED"; tail -30 gpurun_out/ana2/v$v.pytest.log; exit 1; }
  tail -1 gpurun_out/ana2/v$v.pytest.log
  FRS_ANA_V5=$v FRS_ANA_DBG=1 timeout -k 10 200 python -u bench.py --no-extras --no-cpu --queries 0 --steps 2 --warmup 1 > gpurun_out/ana2/dbg$v.json 2> gpurun_out/ana2/dbg$v.err || { tail -20 gpurun_out/ana2/dbg$v.err; exit 1; }
  grep "ana_v5 dbg" gpurun_out/ana2/dbg$v.err | tail -2
done
for v in ${ANA_FORMS:-0 1 2 0 1 2}; do
  FRS_ANA_V5=$v timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/ana2/b$v.json 2> gpurun_out/ana2/b$v.err || { tail -20 gpurun_out/ana2/b$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ana2/b$v.json'));print('v5=$v', d['ms_per_step'], d['kernels_ms'])"
done
if [ -n "$LEVELS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_levels.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/ana2/levels.log 2>&1; rc=$?
  tail -25 gpurun_out/ana2/levels.log
  exit $rc
fi
