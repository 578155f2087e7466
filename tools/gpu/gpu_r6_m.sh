#!/bin/bash
# round 6 call m: branch-free sync-pattern test in the selection pass -- GPU suite, then decode A/B against HEAD's
# selection (variants/libdold.so), alternated on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export FRS_LIB_PATH=$PWD/variants/libdold.so; else unset FRS_LIB_PATH; fi
    timeout -k 10 200 python -u tools/gpu/dec_bench.py 3 300 > $O/$v$r.json 2> $O/$v$r.err || { tail -20 $O/$v$r.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/$v$r.json'))
print('$v', [(b['ms'], b['kernels_ms']) for b in d['batched_decode']], d['bbox_extract']['p50_ms'], d['bbox_extract'].get('kernels_ms_rank0'))"
  done
done
