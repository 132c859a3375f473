# r04 iteration 30: where the dominant-kernel timing sits vs the warm-up steps,
# effect on the driver's 20-step window (A/B, three windows each) and the 2,000-step line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/i30
cd $R && mkdir -p $O
for i in 1 2 3; do for x in 0 1; do BENCH_MEASURE_LAST=$x timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline | sed "s/^/last $x: /" >> $O/window.txt 2>/dev/null || exit $?; done; done
for x in 0 1; do BENCH_MEASURE_LAST=$x timeout -k 10 300 python bench.py --no-cpu-baseline | sed "s/^/last $x: /" >> $O/long.txt 2>/dev/null || exit $?; done
