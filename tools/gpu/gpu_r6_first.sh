#!/bin/bash
# round 6 first call: restore micro, GPU suite + smoke, then the C4 step + C5 + the raw-frames leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 60 ./tools/micro/restore_chain 300 > $O/restore_chain.txt 2>&1 || { cat $O/restore_chain.txt; exit 1; }
cat $O/restore_chain.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --legs raw_frames > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
