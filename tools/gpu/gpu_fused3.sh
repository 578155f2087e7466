#!/bin/bash
# k_fused_v6 forms: timelines (FRS_ANA_DBG records) of the pure fused launch, the hybrid with all tiles analysed
# beforehand (the fused launch as a plain encoder) and the default hybrid; fused parity; C4 step A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fused
tl() {  # name, env...
  local n=$1; shift
  env "$@" FRS_ANA_DBG=1 timeout -k 10 120 python -u bench.py --no-extras --no-cpu --queries 0 --steps 1 --warmup 1 > gpurun_out/fused/tl_$n.json 2> gpurun_out/fused/tl_$n.err || { echo "timeline $n FAILED"; python tools/fused_timeline.py gpurun_out/fused/tl_$n.err; tail -3 gpurun_out/fused/tl_$n.err; return 1; }
  echo "== $n"; python tools/fused_timeline.py gpurun_out/fused/tl_$n.err | head -8
}
tl enc FRS_FUSED=2 FRS_FUSED_K=100000 && tl hyb FRS_FUSED=2 && tl fused FRS_FUSED=1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/fused/p3.log 2>&1 || { echo "fused parity FAILED"; tail -30 gpurun_out/fused/p3.log; exit 1; }
tail -1 gpurun_out/fused/p3.log
for v in ${FORMS:-0 2 1 0 2 1}; do
  FRS_FUSED=$v timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/fused/b$v.json 2> gpurun_out/fused/b$v.err || { tail -20 gpurun_out/fused/b$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fused/b$v.json'));print('fused=$v', d['ms_per_step'], d['kernels_ms'])"
done
