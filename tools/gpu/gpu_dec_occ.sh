#!/bin/bash
# lane-decoder occupancy sweep via FRS_DEC_LANE_LDS (dynamic LDS per 256-thread work-group)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/decocc
for l in ${LDS_LIST:-0 24000 40000 53000 80000}; do
  FRS_DEC_LANE_LDS=$l timeout -k 10 200 python -u tools/gpu/dec_bench.py 2 0 > gpurun_out/decocc/$l.json 2> gpurun_out/decocc/$l.err || { tail -20 gpurun_out/decocc/$l.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/decocc/$l.json'));b=d['batched_decode'][-1];print('lds $l',b['ms'],b['kernels_ms'])"
done
