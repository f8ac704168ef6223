# WaveRNN sample loop: parity tests with two instances, then stamps and timing for one vs two
# instances (FTMI_WR_NI)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/wr_ab; mkdir -p $O
FTMI_WR_NI=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_wavernn.py -x -q --timeout 120 --timeout-method thread > $O/test_ni2.log 2>&1 || exit 1
for ni in 1 2; do
  FTMI_WR_NI=$ni timeout -k 10 120 python tools/wr_stamps.py > $O/stamps_ni$ni.log 2>&1 || exit 1
  FTMI_WR_NI=$ni timeout -k 10 120 python tools/wr_bench.py > $O/bench_ni$ni.log 2>&1 || exit 1
done
echo ALLOK
