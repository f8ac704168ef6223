#!/bin/bash
# A/B several libftmi.so builds (FTMI_LIB) against the in-tree one on the c3 bench, interleaved.
# usage: bash tools/ab_libs.sh "<lib1> <lib2> ..." [rounds] [bench args]
libs=$1; rounds=${2:-2}; shift 2; args="$@"
for i in $(seq $rounds); do
  for v in new $libs; do
    if [ $v = new ]; then unset FTMI_LIB; else export FTMI_LIB=$v; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernels $args 2>gpurun_out/ab.err \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])" || exit 1
    grep -m4 "rnn_bidir" gpurun_out/ab.err | awk '{print "   ", $1, $3}'
  done
done
