#!/bin/bash
# k_fused_v6 with work-group tile claims: parity, then the C4 step for the two-launch form, the hybrid at several K
# and the pure fused launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fused
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/fused/p4.log 2>&1 || { echo "fused parity FAILED"; tail -30 gpurun_out/fused/p4.log; exit 1; }
tail -1 gpurun_out/fused/p4.log
run() {  # label, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/fused/c_$n.json 2> gpurun_out/fused/c_$n.err || { tail -5 gpurun_out/fused/c_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/fused/c_$n.json'));print('$n', d['ms_per_step'], d['kernels_ms'])"
}
run two FRS_FUSED=0 && run hyb4096 FRS_FUSED=2 && run hyb3072 FRS_FUSED=2 FRS_FUSED_K=3072 && run hyb5120 FRS_FUSED=2 FRS_FUSED_K=5120 && run fused FRS_FUSED=1 && run two_b FRS_FUSED=0 && run hyb4096_b FRS_FUSED=2
