#!/bin/bash
# Round-end check on the GPU box: the whole GPU test suite, __graft_entry__.smoke(), and the
# default bench line (what the driver runs).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  tail -${TAILN:-4} gpurun_out/$name.txt
  [ $rc -eq 0 ] || { echo "=== $name FAILED rc=$rc"; exit $rc; }
}
run final_gpu_tests 840 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests
run final_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 run final_bench 400 python -u bench.py
echo ALLOK
