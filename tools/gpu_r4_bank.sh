#!/bin/bash
# Round 4: the c2 prenet bank (channel-halves kernel) — parity tests, then timing and a
# rocprofv3 kernel trace.  Every GPU step under its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "conv_bank" > gpurun_out/r4_bank_tests.txt 2>&1 || { tail -30 gpurun_out/r4_bank_tests.txt; exit 1; }
tail -3 gpurun_out/r4_bank_tests.txt
timeout -k 10 200 python -u tools/bank_bench.py 120 50 halves pairs+finish > gpurun_out/r4_bank_bench.txt 2>&1 || { cat gpurun_out/r4_bank_bench.txt; exit 1; }
cat gpurun_out/r4_bank_bench.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_bank_prof -o prof -- python3 tools/bank_bench.py 120 50 halves pairs+finish > gpurun_out/r4_bank_prof.txt 2>&1 || { tail -20 gpurun_out/r4_bank_prof.txt; exit 1; }
find gpurun_out/r4_bank_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -12'
