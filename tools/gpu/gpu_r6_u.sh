#!/bin/bash
# round 6 call u: the pipe decoder's restore with the group's residuals read up front -- restore micro (forms A-F),
# the C5 / decode GPU tests, then C5 queries tree vs HEAD (variants/libdold.so), alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6u
mkdir -p $O
timeout -k 10 60 ./tools/micro/restore_chain 200
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in tree dold; do
    if [ $v = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/variants/lib$v.so; fi
    timeout -k 10 200 python -u tools/gpu/dec_bench.py 1 1000 > $O/$v$r.json 2> $O/$v$r.err || { tail -20 $O/$v$r.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/$v$r.json'));b=d['bbox_extract']
print('$v', b['p50_ms'], b['p90_ms'], b.get('kernels_ms_rank0'), b['lossless'])"
  done
done
