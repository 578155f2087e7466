#!/bin/bash
# Round-5 closing run: the GPU suite + smoke, then the default bench line (all extras), each bounded; logs under
# gpurun_out/tests and gpurun_out/bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/tests gpurun_out/bench
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=12 > gpurun_out/tests/pytest.log 2>&1 || { tail -40 gpurun_out/tests/pytest.log; exit 1; }
tail -3 gpurun_out/tests/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tests/smoke.log 2>&1 || { cat gpurun_out/tests/smoke.log; exit 1; }
cat gpurun_out/tests/smoke.log
timeout -k 10 480 python -u bench.py > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench.err || { tail -30 gpurun_out/bench/bench.err; exit 1; }
cat gpurun_out/bench/bench.json
