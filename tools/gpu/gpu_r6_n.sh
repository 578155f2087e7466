#!/bin/bash
# round 6 call n: the selection queue (sel_count_queue) -- GPU suite on the tree build, then the batched decode and
# C5 queries for the tree (5 waves/SIMD), dq6 (6 waves/SIMD) and dold (HEAD), alternated on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
FRS_LIB_PATH=$PWD/variants/libdq6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dq6.log 2>&1 || { tail -40 $O/pytest_dq6.log; exit 1; }
tail -1 $O/pytest_dq6.log
for r in 1 2; do
  for v in tree dq6 dold; do
    if [ $v = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/variants/lib$v.so; fi
    timeout -k 10 200 python -u tools/gpu/dec_bench.py 3 300 > $O/$v$r.json 2> $O/$v$r.err || { tail -20 $O/$v$r.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/$v$r.json'))
print('$v', [(b['ms'], b['kernels_ms']['decode']) for b in d['batched_decode']], d['bbox_extract']['p50_ms'], d['bbox_extract'].get('kernels_ms_rank0',{}).get('decode'))"
  done
done
