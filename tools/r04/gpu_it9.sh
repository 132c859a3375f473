# r04 iteration 9: x6 backward probe sweep (timing only), bench window after the
# pre-timing kernel measurement change, K5 / K1 / K4 timelines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for p in 0 8 16 32 56; do D3A_X6_PROBE=$p timeout -k 10 120 python tools/bench_q2.py --x6 | sed "s/^/bwd probe $p: /" >> gpurun_out/i9_probe.txt 2>/dev/null || exit $?; done
for sw in "20 5" "20 5" "2000 50"; do set -- $sw; timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline >> gpurun_out/i9_window.jsonl 2>/dev/null || exit $?; done
export TMPDIR=/tmp
for a in dcql td3bc cqldp; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_$a -o run --output-format csv -- python3 $R/bench.py --algo $a --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_$a.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_$a/run_kernel_trace.csv > gpurun_out/tl_$a.txt; python tools/prof_by_shape.py gpurun_out/tl_$a/run_kernel_trace.csv 70 > gpurun_out/tl_${a}_shape.txt; rm -f gpurun_out/tl_$a/run_kernel_trace.csv
done
