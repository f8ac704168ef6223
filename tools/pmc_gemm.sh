#!/bin/bash
# PMC passes on one GEMM shape, x6 (per-call split) vs x6b (pre-split weights).
# usage: bash tools/pmc_gemm.sh <shape>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
sh=${1:-post.proj1}
mkdir -p gpurun_out/pmc_$sh
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
for v in x6 x6b; do
  pre=""; [ $v = x6b ] && pre="--pre"
  for i in 1 2; do
    eval c=\$C$i
    timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$sh/$v/p$i -- python3 tools/gemm_one.py $sh $pre > gpurun_out/pmc_$sh/$v.p$i.log 2>&1 || { echo "fail $v p$i"; tail -20 gpurun_out/pmc_$sh/$v.p$i.log; exit 3; }
  done
done
echo ok
