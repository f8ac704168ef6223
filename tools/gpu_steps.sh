#!/bin/bash
# Run GPU steps in order, each under its own time limit; continue past ordinary test
# failures (pytest rc 1) but stop at anything else (fault, abort, segfault, timeout).
# usage: tools/gpu_steps.sh "<timeout> <name> <command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  to=${step%% *}; rest=${step#* }; name=${rest%% *}; cmd=${rest#* }
  echo "=== $name (timeout $to s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after $name (rc=$rc)"; exit $rc; fi
done
