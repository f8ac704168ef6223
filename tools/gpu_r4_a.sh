#!/bin/bash
# Round 4: halves-bank phase stamps, then the new GPU tests (TorchScript, split graph,
# compact rerun, K/V workspace after overflow).  Each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
FTMI_LIB=$PWD/forwardtacotron_amd/libftmi_stamps.so timeout -k 10 200 python -u tools/bank_halves_stamps.py 0 1 2 4 3 7 > gpurun_out/r4_halves_stamps.txt 2>&1
rc=$?; cat gpurun_out/r4_halves_stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_model.py -k "torchscript or split_graph or unmarked or compact or timeout or graph or c4_global" \
  tests/test_gpu_fastpitch.py -k "kv_" > gpurun_out/r4_tests_a.txt 2>&1
rc=$?; tail -25 gpurun_out/r4_tests_a.txt; exit $rc
