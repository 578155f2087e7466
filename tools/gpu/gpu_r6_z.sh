#!/bin/bash
# round 6 call z: the C5 restore stores each group while restoring the next -- GPU suite, C5 decode times tree vs HEAD
# (c5_split: host / device output) tree vs HEAD (variants/libdold.so), alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in tree dold tree dold; do
  if [ $v = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/variants/lib$v.so; fi
  timeout -k 10 200 python -u tools/gpu/c5_split.py > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  echo $v; cat $O/$v.json
done
unset FRS_LIB_PATH
timeout -k 10 200 python -u tools/gpu/dec_bench.py 1 1000 > $O/db.json 2> $O/db.err || { tail -20 $O/db.err; exit 1; }
python -c "import json;d=json.load(open('$O/db.json'));b=d['bbox_extract'];print('bench C5', b['p50_ms'], b['p90_ms'], b['kernels_ms_rank0'], b['lossless'])"
