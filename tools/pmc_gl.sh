#!/bin/bash
# PMC passes over the fused Griffin-Lim iteration (tools/gl_bench.py, profiling mode): one
# rocprofv3 run per counter set (the SQ block takes 8 counters a pass)
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_gl
mkdir -p $OUT
export GL_BENCH_PROF=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $OUT/p1 -o run -- python3 $R/tools/gl_bench.py > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p2 -o run -- python3 $R/tools/gl_bench.py > $OUT/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/p3 -o run -- python3 $R/tools/gl_bench.py > $OUT/p3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/p4 -o run -- python3 $R/tools/gl_bench.py > $OUT/p4.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/tools/gl_bench.py > $OUT/kt.log 2>&1
echo done
