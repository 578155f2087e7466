#!/bin/bash
# round 6 call g: encoder A/B -- tree vs variants/libeA.so (one barrier per ticket), alternating, C4 step only
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 300 env FRS_LIB_PATH=$PWD/variants/libeA.so python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_stereo.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_eA.log 2>&1 || { tail -30 $O/pytest_eA.log; exit 1; }
tail -2 $O/pytest_eA.log
for lib in tree variants/libeA.so tree variants/libeA.so tree variants/libeA.so; do
  if [ "$lib" = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-extras --queries 0 --steps 20 > $O/ab.json 2> $O/ab.err || { tail -30 $O/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ab.json'));print('$lib', d['ms_per_step'], d['kernels_ms'])"
done
