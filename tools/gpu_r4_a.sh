#!/bin/bash
# Round 4: halves-bank phase stamps, recurrence phase stamps + no-wait step time, then the
# new GPU tests (TorchScript, split graph, compact rerun, K/V workspace after overflow, c4).
# Each GPU step under its own limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  tail -30 gpurun_out/$name.txt
  [ $rc -eq 0 ] || { echo "=== $name FAILED rc=$rc"; exit $rc; }
}
export FTMI_LIB_STAMPS=$PWD/forwardtacotron_amd/libftmi_stamps.so
run r4_halves_stamps 200 env FTMI_LIB=$FTMI_LIB_STAMPS python -u tools/bank_halves_stamps.py 0 1 2 4 3 7
run r4_rnn_stamps 300 env FTMI_LIB=$FTMI_LIB_STAMPS python -u tools/rnn_stamps.py
run r4_rnn_diag 400 env DIAG_VALS="0 2 0 2" python -u tools/rnn_diag.py
run r4_tests_a 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_model.py -k "torchscript or split_graph or unmarked or compact or timeout or graph or c4_global" \
  tests/test_gpu_fastpitch.py -k "kv_"
echo ALLOK
