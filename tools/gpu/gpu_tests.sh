#!/bin/bash
# GPU parity suite (every -m gpu test, one process) + smoke; logs under gpurun_out/tests/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/tests
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=12 ${PYTEST_ARGS:-} > gpurun_out/tests/pytest.log 2>&1 || { tail -40 gpurun_out/tests/pytest.log; exit 1; }
tail -3 gpurun_out/tests/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tests/smoke.log 2>&1 || { cat gpurun_out/tests/smoke.log; exit 1; }
cat gpurun_out/tests/smoke.log
