#!/bin/bash
# PMC passes on one GEMM shape for two settings of one switch.
# usage: bash tools/pmc_gemm_env.sh <shape> <ENV> <v0> <v1>; then python tools/pmc_summary.py <dir>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
sh=$1; env=$2
mkdir -p gpurun_out/pmc_$sh
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
for v in $3 $4; do
  for i in 1 2; do
    eval c=\$C$i
    export $env=$v
    timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$sh/v$v/p$i -- python3 tools/gemm_one.py $sh --pre > gpurun_out/pmc_$sh/v$v.p$i.log 2>&1 || { echo "fail $v p$i"; tail -20 gpurun_out/pmc_$sh/v$v.p$i.log; exit 3; }
  done
done
echo ok
