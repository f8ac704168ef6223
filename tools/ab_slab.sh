for i in 1 2; do
for v in 0 8589934592; do
  FTMI_GEMM_SLAB_MIN=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('min=$v', d['ms_per_step'])"
done
done
