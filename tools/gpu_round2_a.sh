set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "rnn or lstm or gru" -x -q --timeout 120 --timeout-method thread > gpurun_out/k.log 2>&1 || { echo KFAIL; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/k.log 2>&1 || { echo MFAIL; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --kernels --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
FTMI_RNN_ROWS=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --kernels --no-cpu-baseline > gpurun_out/bench_c3_ks.json 2> gpurun_out/bench_c3_ks.err || exit 1
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --kernels --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
FTMI_RNN_ROWS=0 timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --kernels --no-cpu-baseline > gpurun_out/bench_c2_ks.json 2> gpurun_out/bench_c2_ks.err || exit 1
echo ALLOK
