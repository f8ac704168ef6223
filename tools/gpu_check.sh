# model-level GPU checks + c3 / c2 bench lines (no CPU baseline), for A/B after a change
set -o pipefail
mkdir -p gpurun_out/chk
O=gpurun_out/chk
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_accuracy.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernels > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python bench.py --config c2 --callbacks gen_forward --steps 30 --warmup 3 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
python - <<'PY'
import json
for c in ('c3', 'c2'):
    d = json.loads(open(f'gpurun_out/chk/{c}.json').read().strip().splitlines()[-1])
    print(c, d['ms_per_step'], 'ms', d['value'], d['parity'] if 'parity' in d else '', d.get('host_to_host', {}).get('ms_per_step'))
PY
