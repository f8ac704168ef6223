# c2 evidence refresh: the bench line as gen_forward.py calls generate() (with the per-kernel
# table), the Griffin-Lim sentence step beside it, and the rocprofv3 kernel-trace summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-c2}
mkdir -p $O
timeout -k 10 300 python bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --kernels --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python bench.py --config c2 --callbacks gen_forward --vocoder griffinlim --steps 20 --warmup 3 > $O/bench_c2_gl.json 2> $O/bench_c2_gl.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 10 --warmup 3 --no-cpu-baseline --no-host-loop > $O/prof_c2.log 2>&1 || exit 1
echo ALLOK
