set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "conv_bank" -x -q --timeout 120 --timeout-method thread > gpurun_out/bank.log 2>&1 || { echo BANKFAIL; exit 1; }
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-host-loop > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
FTMI_BANK_BALANCED=0 timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-host-loop > gpurun_out/bench_c2_unbal.json 2> gpurun_out/bench_c2_unbal.err || exit 1
echo ALLOK
