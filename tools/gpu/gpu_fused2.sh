#!/bin/bash
# k_fused_v6 timeline (per-work-group phase times) + parity of the fused tests + the C4 step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fused
FRS_FUSED=1 FRS_ANA_DBG=1 timeout -k 10 120 python -u bench.py --no-extras --no-cpu --queries 0 --steps 1 --warmup 1 > gpurun_out/fused/tl.json 2> gpurun_out/fused/tl.err || { python tools/fused_timeline.py gpurun_out/fused/tl.err; tail -3 gpurun_out/fused/tl.err; exit 1; }
python tools/fused_timeline.py gpurun_out/fused/tl.err
FRS_FUSED=1 timeout -k 10 120 python -u bench.py --no-extras --no-cpu --queries 0 --steps 3 --warmup 1 > gpurun_out/fused/q.json 2> gpurun_out/fused/q.err || { echo "fused bench FAILED"; tail -5 gpurun_out/fused/q.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/fused/q.json'));print('fused quick', d['ms_per_step'], d['kernels_ms'])"
FRS_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/fused/p2.log 2>&1 || { echo "fused parity FAILED"; tail -30 gpurun_out/fused/p2.log; exit 1; }
tail -1 gpurun_out/fused/p2.log
for v in ${FORMS:-0 1 0 1}; do
  FRS_FUSED=$v timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/fused/b$v.json 2> gpurun_out/fused/b$v.err || { tail -20 gpurun_out/fused/b$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fused/b$v.json'));print('fused=$v', d['ms_per_step'], d['kernels_ms'])"
done
