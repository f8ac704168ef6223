# A/B of the f16x3 split-row hand-offs (FTMI_SPLIT_ROWS / FTMI_SPLIT_BANK_IN) on one box, c3
set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
  for v in 11 10 00; do
    FTMI_SPLIT_ROWS=${v:0:1} FTMI_SPLIT_BANK_IN=${v:1:1} timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernels > gpurun_out/ab/c3_$v.$i.json 2> gpurun_out/ab/c3_$v.$i.err || exit 1
    python - "$v" "$i" <<'PY'
import json, sys
v, i = sys.argv[1:]
d = json.loads(open(f'gpurun_out/ab/c3_{v}.{i}.json').read().strip().splitlines()[-1])
ks = [l for l in open(f'gpurun_out/ab/c3_{v}.{i}.err') if 'conv_bank' in l or 'K=6144' in l or 'K=12288' in l or 'split_rows' in l]
print(v, i, d['ms_per_step'], ' | '.join(' '.join(l.split()[:1] + l.split()[2:3]) for l in ks), flush=True)
PY
  done
done
