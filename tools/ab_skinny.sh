#!/bin/bash
# A/B the in-tree libftmi.so against a baseline build on the batch-1 skinny GEMM shapes
# (c2 prenet bank + proj1), interleaved.  usage: bash tools/ab_skinny.sh <base.so> [rounds]
base=$1; rounds=${2:-3}
mkdir -p gpurun_out
for i in $(seq $rounds); do
  for v in new base; do
    if [ $v = base ]; then export FTMI_LIB=$base; else unset FTMI_LIB; fi
    echo -n "$v: "
    timeout -k 10 100 python tools/skinny_bench.py skinnycpb=2 2>gpurun_out/ab_skinny_$v.err || exit 1
  done
done
# the c2 step (batch 1: the skinny kernel's caller), interleaved
for i in $(seq $rounds); do
  for v in new base; do
    if [ $v = base ]; then export FTMI_LIB=$base; else unset FTMI_LIB; fi
    timeout -k 10 200 python bench.py --config c2 --callbacks gen_forward --steps 30 --warmup 5 --no-cpu-baseline --no-host-loop 2>gpurun_out/ab_c2_$v.err \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v c2', d['ms_per_step'], d['prenet_bank']['avg_launch_ms'])" || exit 1
  done
done
