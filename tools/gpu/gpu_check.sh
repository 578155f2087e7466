#!/bin/bash
# Re-entry check: smoke, GPU parity suite, one default-size bench line (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/check/pytest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/check/bench.log 2>&1 || exit 1
echo done
