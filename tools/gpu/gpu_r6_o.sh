#!/bin/bash
# round 6 call o: one-wave work-groups for the batched lane decoder (tree) vs 4-wave groups (dw4) vs HEAD (dold)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
FRS_LIB_PATH=$PWD/variants/libdw4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dw4.log 2>&1 || { tail -40 $O/pytest_dw4.log; exit 1; }
tail -1 $O/pytest_dw4.log
for r in 1 2; do
  for v in tree dw4 dold; do
    if [ $v = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/variants/lib$v.so; fi
    timeout -k 10 200 python -u tools/gpu/dec_bench.py 3 300 > $O/$v$r.json 2> $O/$v$r.err || { tail -20 $O/$v$r.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/$v$r.json'))
print('$v', [(b['ms'], b['kernels_ms']['decode_frames']) for b in d['batched_decode']], d['bbox_extract']['p50_ms'], d['bbox_extract'].get('kernels_ms_rank0',{}).get('decode'))"
  done
done
