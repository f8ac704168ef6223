#!/bin/bash
# One measurement round of the c2 prenet bank (run on the GPU box through gpurun): the bank
# kernel tests, phase stamps of the given variants (tools/bank_halves_stamps.py names:
# img, img:<diag bits>, ...), HIP-graph timing (tools/bank_bench.py), then the c2 bench
# line.  Stops at the first failure.  usage: TAG=r4n bash tools/gpu_bank_round.sh [variant ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-bank}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  tail -${TAILN:-6} gpurun_out/$name.txt
  [ $rc -eq 0 ] || { echo "=== $name FAILED rc=$rc"; exit $rc; }
}
run ${T}_bank_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv_bank"
TAILN=40 run ${T}_stamps 200 env SLOWEST=4 FTMI_LIB=$PWD/forwardtacotron_amd/libftmi_stamps.so python -u tools/bank_halves_stamps.py ${@:-img}
run ${T}_bank_bench 200 python -u tools/bank_bench.py 120 50 halves-image halves
TAILN=1 run ${T}_c2 300 python -u bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --no-cpu-baseline
echo ALLOK
