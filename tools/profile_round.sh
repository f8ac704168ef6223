#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box through gpurun):
#   1. --kernel-trace --stats on the default bench command (per-kernel durations)
#   2. PMC passes FETCH_SIZE and WRITE_SIZE (separate passes, kernel-trace only) for HBM traffic
# usage: bash tools/profile_round.sh <tag> [extra bench args]
set -u
tag=${1:-r1}; shift || true
out=gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
run trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@"
run fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@"
run write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@"
echo done
