#!/bin/bash
# A/B one environment variable on the c3 bench in one box session, interleaved rounds.
# usage: bash tools/ab_env.sh VAR "val1 val2 ..." [rounds]
var=$1; vals=$2; rounds=${3:-2}
for i in $(seq $rounds); do
  for v in $vals; do
    env $var=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$var=$v', d['ms_per_step'])"
  done
done
