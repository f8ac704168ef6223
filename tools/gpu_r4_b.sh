#!/bin/bash
# Round 4: slab-prologue probe, then the new model GPU tests.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  tail -${TAILN:-30} gpurun_out/$name.txt
  [ $rc -eq 0 ] || { echo "=== $name FAILED rc=$rc"; exit $rc; }
}
run r4_probe_slab 120 ./tools/probe_slab.bin
run r4_tests_b 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_model.py -k "torchscript or split_graph or unmarked or compact or timeout or graph or c4_global"
echo ALLOK
