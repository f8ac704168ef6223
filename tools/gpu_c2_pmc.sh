# c2 traffic evidence: kernel trace + FETCH_SIZE / WRITE_SIZE passes of the c2 bench
# (tools/profile_round.sh), condensed (tools/summarize_prof.py), then the c2 bench line that
# reads them; the condensed files are copied under gpurun_out/ to come back.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh r2c2 --config c2 --callbacks gen_forward > gpurun_out/prof_r2c2.log 2>&1 || exit 1
python tools/summarize_prof.py gpurun_out/prof_r2c2 r2c2 || exit 1
mkdir -p gpurun_out/c2pmc && cp profiles/r2c2_kernel_stats.csv profiles/r2c2_pmc_traffic.json gpurun_out/c2pmc/ || exit 1
timeout -k 10 300 python bench.py --config c2 --callbacks gen_forward --steps 20 --warmup 3 --kernels > gpurun_out/c2pmc/bench_c2.json 2> gpurun_out/c2pmc/bench_c2.err || exit 1
echo ALLOK
