#!/bin/bash
# A/B the in-tree libftmi.so against a baseline build (FTMI_LIB=<path>) on the c3 bench in
# one box session, interleaved rounds.  usage: bash tools/ab_lib.sh <base.so> [rounds] [bench args]
base=$1; rounds=${2:-3}; shift 2; args="$@"
for i in $(seq $rounds); do
  for v in new base; do
    if [ $v = base ]; then export FTMI_LIB=$base; else unset FTMI_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernels $args 2>gpurun_out/ab_$v.err \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])" || exit 1
    grep -m3 "rnn_bidir" gpurun_out/ab_$v.err | awk '{print "   ", $1, $3}'
  done
done
