#!/bin/bash
# Round 4: bank tests + stamps of the final halves kernel, then the round's bench lines
# (tools/gpu_r4_measure.sh bench).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  tail -${TAILN:-6} gpurun_out/$name.txt
  [ $rc -eq 0 ] || { echo "=== $name FAILED rc=$rc"; exit $rc; }
}
run r4h_bank_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv_bank"
run r4h_stamps 200 env FTMI_LIB=$PWD/forwardtacotron_amd/libftmi_stamps.so python -u tools/bank_halves_stamps.py img img:256 img:32
OUT=r4 bash tools/gpu_r4_measure.sh bench || exit $?
echo ALLOK
