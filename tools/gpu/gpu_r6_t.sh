#!/bin/bash
# round 6 call t: analysis chunk size -- C4 step with the plain 64-sample form (tree default), the 32-sample
# prefetching form (FRS_ANA_PF=1), the plain 32-sample form (variants/liba32.so), alternated; C3 with the tree's
# prefetch (32-sample) against HEAD's (64-sample, variants/libahead.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_encode_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
FRS_LIB_PATH=$PWD/variants/liba32.so timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_encode_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest_a32.log 2>&1 || { tail -40 $O/pytest_a32.log; exit 1; }
tail -1 $O/pytest_a32.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-extras --no-cpu --queries 0 --steps 10 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], d['kernels_ms'])"
}
for r in 1 2; do
  run plain$r FRS_ANA_PF=0
  run pf32_$r FRS_ANA_PF=1
  run a32_$r FRS_LIB_PATH=$PWD/variants/liba32.so FRS_ANA_PF=0
done
for r in 1 2; do
  for v in tree ahead; do
    if [ $v = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/variants/libahead.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --queries 0 --legs c3_streaming > $O/c3$v$r.json 2> $O/c3$v$r.err || { tail -20 $O/c3$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c3$v$r.json'));c=d['c3_streaming'];print('c3 $v', c['ms_per_step'], c['kernels_ms'])"
  done
done
