#!/bin/bash
# round 5 first call: GPU suite + smoke, then the C4 step alone (no extras)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r5a/pytest.log 2>&1 || { tail -40 gpurun_out/r5a/pytest.log; exit 1; }
tail -3 gpurun_out/r5a/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5a/smoke.log 2>&1 || { cat gpurun_out/r5a/smoke.log; exit 1; }
cat gpurun_out/r5a/smoke.log
timeout -k 10 300 python -u bench.py --no-extras --no-cpu --queries 200 --steps 20 > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || { tail -30 gpurun_out/r5a/bench.err; exit 1; }
cat gpurun_out/r5a/bench.json
