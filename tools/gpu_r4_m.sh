#!/bin/bash
# Round 4: the pair bank (proj1 finishes the halves) — kernel + model tests, then the c2
# bench line (bank plus finishing work, and the in-kernel-finish A/B).  Stops at the first
# failure.
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
run r4m_bank_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv_bank or conv1d"
run r4m_model_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_accuracy.py
TAILN=1 run r4m_c2 300 python -u bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --no-cpu-baseline
echo ALLOK
