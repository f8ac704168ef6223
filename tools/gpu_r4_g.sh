#!/bin/bash
# Round 4: halves bank with per-wave arrival counters — bank tests, stamps, timing, the c2
# bench line (image vs planes A/B in the same process), then the whole GPU test suite.
# Stops at the first failure.
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
run r4g_bank_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv_bank"
run r4g_stamps 200 env FTMI_LIB=$PWD/forwardtacotron_amd/libftmi_stamps.so python -u tools/bank_halves_stamps.py img img:256 img:32
run r4g_bank_bench 200 python -u tools/bank_bench.py 120 50 halves-image halves
TAILN=1 run r4g_c2 300 python -u bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --no-cpu-baseline
run r4g_gpu_tests 840 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests
echo ALLOK
