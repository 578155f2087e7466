#!/bin/bash
# SQ counters of the encoder kernel per environment setting (two 8-counter passes each), summarised per kernel
# usage: ENVS="FRS_ENC_V=3 FRS_ENC_V=4" ./tools/gpu/gpu_sq_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/sqab; mkdir -p gpurun_out/sqab
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-extras --queries 0"
i=0
for e in ${ENVS:-FRS_ENC_V=3 FRS_ENC_V=4}; do
  i=$((i+1))
  export ${e%%=*}=${e#*=}
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/sqab/$i/a -o run -- $B > gpurun_out/sqab/$i.a.log 2>&1 || { tail -5 gpurun_out/sqab/$i.a.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/sqab/$i/b -o run -- $B > gpurun_out/sqab/$i.b.log 2>&1 || { tail -5 gpurun_out/sqab/$i.b.log; exit 1; }
  unset ${e%%=*}
  echo "== $e"
  python3 tools/pmc_by_kernel.py gpurun_out/sqab/$i/a gpurun_out/sqab/$i/b -k k_encode
done
