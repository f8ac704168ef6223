#!/bin/bash
# Interleaved c3 sweep of environment switches against the defaults.
# usage: bash tools/ab_env_sweep_c3.sh [rounds] "VAR=value" ...
rounds=$1; shift
for i in $(seq $rounds); do
  for e in default "$@"; do
    if [ "$e" = default ]; then pre=""; else pre="env $e"; fi
    $pre timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-loop 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$e', d['ms_per_step'])" || exit 1
  done
done
