#!/bin/bash
# Parity suite + bench, then LDS/VALU counters of the encode path per FRS_ABLATE setting
# (0 full, 2 no CRC, 4 no Rice packing, 16 no arena stores, 23 core only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/lds; mkdir -p gpurun_out/lds
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lds/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/lds/bench.log 2>&1 || exit 1
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --queries 0"
for a in 0 2 4 16 23; do
  FRS_ABLATE=$a timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/lds/a$a -o run -- $B > gpurun_out/lds/a$a.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/lds/a$a > gpurun_out/lds/sum$a.md
done
echo done
