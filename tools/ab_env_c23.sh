#!/bin/bash
# A/B an environment switch on the c3 and c2 benches, interleaved.
# usage: bash tools/ab_env_c23.sh "VAR=value" [rounds]
envset=$1; rounds=${2:-3}
for i in $(seq $rounds); do
  for v in new base; do
    for c in c3 c2; do
      if [ $c = c2 ]; then a="--config c2 --callbacks gen_forward --steps 30 --warmup 5"; else a="--steps 10 --warmup 3"; fi
      if [ $v = base ]; then pre="env $envset"; else pre=""; fi
      $pre timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-host-loop 2>/dev/null \
        | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v $c', d['ms_per_step'])" || exit 1
    done
  done
done
