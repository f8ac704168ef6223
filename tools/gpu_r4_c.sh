#!/bin/bash
# Round 4: halves bank after the address-arithmetic rework — parity tests, phase stamps,
# timing (graph / eager / cold) and a rocprofv3 kernel trace.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  tail -${TAILN:-12} gpurun_out/$name.txt
  [ $rc -eq 0 ] || { echo "=== $name FAILED rc=$rc"; exit $rc; }
}
run r4c_bank_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv_bank or conv1d or highway or f16x3_range or split_rows"
run r4c_stamps 200 env FTMI_LIB=$PWD/forwardtacotron_amd/libftmi_stamps.so python -u tools/bank_halves_stamps.py 0 8 128 136
run r4c_bank_bench 200 python -u tools/bank_bench.py 120 50 halves pairs+finish

run r4c_bank_prof 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c_prof -o run -- python3 tools/bank_bench.py 120 50 halves pairs+finish
find gpurun_out/r4c_prof -name "*kernel_stats.csv" -exec head -6 {} \;
echo ALLOK
