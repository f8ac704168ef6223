cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sbp
timeout -k 10 120 python tools/skinny_bench.py > gpurun_out/sb.log 2>&1 || exit $?
for c in skinnycpb=2 unbalancedcpb=2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sbp/$c -- python3 tools/skinny_bench.py $c > gpurun_out/sbp/$c.log 2>&1 || exit $?
done
echo done
