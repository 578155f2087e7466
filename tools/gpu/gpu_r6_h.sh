#!/bin/bash
# round 6 call h: the full suite with the one-barrier encoder in the tree; C4 step; persistent k_sync_count without
# prefetch (FRS_SYNC_P=1) against the per-block launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --no-extras --steps 20 > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
python -c "import json;d=json.load(open('$O/c4.json'));print(d['ms_per_step'], d['kernels_ms'], d['bbox_extract']['p50_ms'])"
for sp in 1 0 1 0; do
  export FRS_SYNC_P=$sp
  timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --queries 0 --legs batched_decode > $O/dec.json 2> $O/dec.err || { tail -30 $O/dec.err; exit 1; }
  python -c "import json;d=json.load(open('$O/dec.json'));print('SYNC_P=$sp', json.dumps(d['batched_decode']))"
done
