#!/bin/bash
# Round 4: halves bank stamps with per-XCD start / end spread (img) and without the partner
# exchange (img:4, timing only), plus bank_bench HIP-graph timing of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SLOWEST=4 timeout -k 10 200 env FTMI_LIB=$PWD/forwardtacotron_amd/libftmi_stamps.so python -u tools/bank_halves_stamps.py img img:4 > gpurun_out/r4l_stamps.txt 2>&1 || { tail -5 gpurun_out/r4l_stamps.txt; exit 1; }
cat gpurun_out/r4l_stamps.txt
timeout -k 10 200 env FTMI_BANK_HALVES_DIAG=4 python -u tools/bank_bench.py 120 50 halves-image > gpurun_out/r4l_bench.txt 2>&1 || { tail -5 gpurun_out/r4l_bench.txt; exit 1; }
cat gpurun_out/r4l_bench.txt
echo ALLOK
