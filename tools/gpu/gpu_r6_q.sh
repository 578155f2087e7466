#!/bin/bash
# round 6 call q: the prefix-CRC count pass in the queue form -- GPU suite (incl. the pcrc tests), then the batched
# C4 decode with the reading span check (default) and the prefix-CRC one (FRS_SPAN_READ=2), alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
FRS_SPAN_READ=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pcrc.log 2>&1 || { tail -40 $O/pytest_pcrc.log; exit 1; }
tail -1 $O/pytest_pcrc.log
for r in 1 2; do
  for v in read pcrc; do
    if [ $v = pcrc ]; then export FRS_SPAN_READ=2; else unset FRS_SPAN_READ; fi
    timeout -k 10 200 python -u tools/gpu/dec_bench.py 3 0 > $O/$v$r.json 2> $O/$v$r.err || { tail -20 $O/$v$r.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/$v$r.json'))
print('$v', [(b['ms'], b['kernels_ms']) for b in d['batched_decode']])"
  done
done
timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --queries 0 --legs convert_multiband > $O/mb.json 2> $O/mb.err || { tail -20 $O/mb.err; exit 1; }
python -c "import json;d=json.load(open('$O/mb.json'));print(json.dumps(d['convert_multiband']['decode']))"
