# WaveRNN sample loop: stamps and timing for one vs two instances (FTMI_WR_NI)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/wr_ab; mkdir -p $O
for ni in 1 2; do
  FTMI_WR_NI=$ni timeout -k 10 120 python tools/wr_stamps.py > $O/stamps_ni$ni.log 2>&1 || exit 1
  FTMI_WR_NI=$ni timeout -k 10 120 python tools/wr_bench.py > $O/bench_ni$ni.log 2>&1 || exit 1
done
echo ALLOK
