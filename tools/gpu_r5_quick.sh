#!/bin/bash
# Round 5, quick GPU check of this round's new kernels (spread CBHG tail, U = 8 and
# one-barrier recurrences), then the recurrence timing sweep.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "spread or lstm_through or f16x3_kernels" \
  > gpurun_out/r5_quick_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/r5_quick_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5_rnn_diag.sh
