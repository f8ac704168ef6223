# Round-2 measurement: default bench lines (c3 with cpu_baseline, c2 as gen_forward calls it,
# c5 FastPitch), rocprofv3 kernel-trace summaries of the c3 / c2 / c5 benches and the PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the c3 bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r2}
mkdir -p $O
timeout -k 10 400 python bench.py --kernels > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --kernels --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python bench.py --model fast_pitch --steps 10 --warmup 3 --kernels --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-loop > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 10 --warmup 3 --no-cpu-baseline --no-host-loop > $O/prof_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --model fast_pitch --steps 5 --warmup 2 --no-cpu-baseline --no-host-loop > $O/prof_c5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop > $O/fetch_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop > $O/write_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_wr -o run -- python3 bench.py --model wavernn --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_wr.log 2>&1 || exit 1
echo ALLOK
