#!/bin/bash
# Round 4: the slab kernels' column-band tile order (FTMI_SLAB_BAND): parity with the band
# order, then per-shape kernel time (rocprofv3 stats) and L2->fabric read bytes (FETCH_SIZE)
# with band 0 (the XCD-aware row-tile order) and 2.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > gpurun_out/r4d/$name.txt 2>&1
  local rc=$?
  tail -${TAILN:-4} gpurun_out/r4d/$name.txt
  [ $rc -eq 0 ] || { echo "=== $name FAILED rc=$rc"; exit $rc; }
}
run tests_band2 600 env FTMI_SLAB_BAND=2 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv1d or conv_bank or slab_prefetch or highway"
for shape in fp.conv1 post.bank post.proj1 pre.bank lstm_in; do
  for b in 0 2; do
    run stats_${shape}_b$b 120 env FTMI_SLAB_BAND=$b rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d/stats_${shape}_b$b -o run -- python3 tools/gemm_one.py $shape --pre --iters 20
    grep -h "slab" gpurun_out/r4d/stats_${shape}_b$b/run_kernel_stats.csv | cut -d, -f1-4 | head -2
  done
done
for b in 0 2; do
  run fetch_fp_b$b 120 env FTMI_SLAB_BAND=$b rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4d/fetch_fp_b$b -o run -- python3 tools/gemm_one.py fp.conv1 --pre --iters 5
done
echo ALLOK
