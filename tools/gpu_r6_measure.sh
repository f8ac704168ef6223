#!/bin/bash
# Round-6 measurement on the GPU box: bench lines (c3, c2 as gen_forward calls it, c2 +
# Griffin-Lim, c5 FastPitch + Griffin-Lim with its HIP STFT kernels, WaveRNN), rocprofv3
# kernel-trace summaries, PMC traffic passes (FETCH_SIZE / WRITE_SIZE: separate runs) and the
# MFMA-busy pass.  usage: OUT=r6 bash tools/gpu_r5_measure.sh [bench|prof|pmc|mfma|all]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6}
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
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
if [ "$PART" = bench ] || [ "$PART" = all ]; then
  step bench_c3 400 python bench.py --steps 20 --warmup 3 --kernels
  step bench_c2 300 python bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --kernels
  step bench_c2_gl 400 python bench.py --config c2 --callbacks gen_forward --vocoder griffinlim --nnls lbfgsb --vocoder-steps 3 --steps 20 --warmup 3 --no-cpu-baseline
  step bench_c2_gl_fista 300 python bench.py --config c2 --callbacks gen_forward --vocoder griffinlim --nnls fista --steps 20 --warmup 3 --no-cpu-baseline
  step bench_c5 500 python bench.py --model fast_pitch --vocoder griffinlim --nnls fista --steps 10 --warmup 3 --kernels
  step bench_wr 300 python bench.py --model wavernn --steps 3 --warmup 1
fi
if [ "$PART" = prof ] || [ "$PART" = all ]; then
  step prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-loop
  step prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 10 --warmup 3 --no-cpu-baseline --no-host-loop
  step prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --model fast_pitch --vocoder griffinlim --nnls fista --steps 3 --warmup 2 --no-cpu-baseline --no-host-loop
fi
if [ "$PART" = pmc ] || [ "$PART" = all ]; then
  step fetch_c3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
  step write_c3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
  step fetch_c2 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 3 --warmup 2 --no-cpu-baseline --no-host-loop
  step write_c2 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 3 --warmup 2 --no-cpu-baseline --no-host-loop
  step fetch_c5 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5 -o run -- python3 bench.py --model fast_pitch --vocoder griffinlim --nnls fista --steps 1 --warmup 1 --no-cpu-baseline --no-host-loop
  step write_c5 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5 -o run -- python3 bench.py --model fast_pitch --vocoder griffinlim --nnls fista --steps 1 --warmup 1 --no-cpu-baseline --no-host-loop
fi
if [ "$PART" = mfma ] || [ "$PART" = all ]; then
  step mfma_c3 300 rocprofv3 --pmc $MF --output-format csv -d $O/mfma_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
  step mfma_c2 300 rocprofv3 --pmc $MF --output-format csv -d $O/mfma_c2 -o run -- python3 bench.py --config c2 --callbacks gen_forward --steps 3 --warmup 2 --no-cpu-baseline --no-host-loop
  step mfma_c5 400 rocprofv3 --pmc $MF --output-format csv -d $O/mfma_c5 -o run -- python3 bench.py --model fast_pitch --steps 2 --warmup 1 --no-cpu-baseline --no-host-loop
fi
if [ "$PART" = c4 ]; then  # the N > 1 path: RCCL tests at world 1, gloo rehearsal at world 2 on one GPU
  step c4_tests 300 python -u -m pytest tests/test_sharded.py -m gpu -x -v --timeout 200 --timeout-method thread
  step c4_gloo2 500 env FTMI_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-host-loop
  step c4_gloo2_pipe 500 env FTMI_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --no-host-loop --gather-overlap on
fi
echo ALLOK
