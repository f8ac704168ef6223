# Round-4 measurement (run on the GPU box through gpurun): the bench lines of every config
# with their CPU baselines (c3, c2 as gen_forward calls it, c2 with the Griffin-Lim vocoder,
# c5 FastPitch, the WaveRNN vocoder), rocprofv3 kernel-trace summaries of the c3 / c2 / c5 /
# WaveRNN benches, and the PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) of
# c3 and c2.  usage: OUT=r4 bash tools/gpu_r4_measure.sh [part]   part: bench | prof | pmc | all
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r4}
PART=${1:-all}
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "=== $name FAILED rc=$rc"; tail -5 $O/$name.err; exit $rc; fi
  tail -c 300 $O/$name.out; echo
}
if [ "$PART" = bench ] || [ "$PART" = all ]; then
  step bench_c3 400 python bench.py --steps 20 --warmup 3 --kernels
  step bench_c2 300 python bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --kernels
  step bench_c2_gl 300 python bench.py --config c2 --callbacks gen_forward --vocoder griffinlim --steps 20 --warmup 3 --no-cpu-baseline
  step bench_c5 400 python bench.py --model fast_pitch --steps 10 --warmup 3 --kernels
  step bench_wr 300 python bench.py --model wavernn --steps 3 --warmup 1
fi
if [ "$PART" = prof ] || [ "$PART" = all ]; then
  step prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-loop
  step prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 10 --warmup 3 --no-cpu-baseline --no-host-loop
  step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --model fast_pitch --steps 5 --warmup 2 --no-cpu-baseline --no-host-loop
  step prof_wr 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_wr -o run -- python3 bench.py --model wavernn --steps 2 --warmup 1 --no-cpu-baseline
fi
if [ "$PART" = pmc ] || [ "$PART" = all ]; then
  step fetch_c3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
  step write_c3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
  step fetch_c5 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5 -o run -- python3 bench.py --model fast_pitch --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
  step write_c5 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5 -o run -- python3 bench.py --model fast_pitch --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
  step fetch_c2 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 3 --warmup 2 --no-cpu-baseline --no-host-loop
  step write_c2 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 3 --warmup 2 --no-cpu-baseline --no-host-loop
fi
echo ALLOK
