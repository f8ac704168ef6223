# GEMV recurrence checks: recurrence kernel tests, model tests, c2 A/B (GEMV on / off)
set -o pipefail
mkdir -p gpurun_out/chk
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "rnn or gru or lstm" --timeout 120 --timeout-method thread > gpurun_out/chk/k.log 2>&1 || { echo KFAIL; tail -30 gpurun_out/chk/k.log; exit 1; }
tail -1 gpurun_out/chk/k.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_accuracy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/chk/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/chk/tests.log; exit 1; }
tail -1 gpurun_out/chk/tests.log
for g in 1 0 1; do FTMI_RNN_GEMV=$g timeout -k 10 200 python bench.py --config c2 --callbacks gen_forward --steps 30 --warmup 3 --no-cpu-baseline --kernels > gpurun_out/chk/c2_$g.json 2> gpurun_out/chk/c2_$g.err || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/chk/c2_$g.json').read().strip().splitlines()[-1]); print('gemv=$g', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"; done
