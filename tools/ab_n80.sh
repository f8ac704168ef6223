# A/B of the narrow-GEMM change (x6b skips column tiles past N) against ab/libftmi_base.so:
# the three c3 N = 80 shapes, then the c3 bench, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_n80; mkdir -p $O
for i in 1 2; do
  timeout -k 10 100 python tools/n80_bench.py > $O/new_$i.log 2>&1 || exit 1
  FTMI_LIB=ab/libftmi_base.so timeout -k 10 100 python tools/n80_bench.py > $O/base_$i.log 2>&1 || exit 1
done
bash tools/ab_lib.sh ab/libftmi_base.so 2 > $O/c3_ab.log 2>&1 || exit 1
echo ALLOK
