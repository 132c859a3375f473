#!/bin/bash
# round 6 final: full GPU suite, smoke, every bench line (K2 with its CPU
# baseline; bf16, K4, repro, K1, K3, K5), the rocprof kernel-trace summary of
# the default bench command.  Outputs under gpurun_out/r6final/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6final
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
# the arbiter's per-tensor margins (HIP vs fp64 on HIP's ReLU decisions, the bar)
timeout -k 10 400 python -u -m pytest -s -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_cql_parity.py tests/test_gpu_arbiters.py tests/test_gpu_dp.py tests/test_gpu_production_path.py tests/test_gpu_sac_parity.py > $O/arbiter_margins.log 2>&1 || { tail -30 $O/arbiter_margins.log; exit 1; }
tail -1 $O/arbiter_margins.log
timeout -k 10 300 python bench.py > $O/bench_cql.json 2> $O/bench_cql.err || { tail -20 $O/bench_cql.err; exit 1; }
for spec in "cql --precision bf16:cql_bf16" "cqldp:cqldp" "cqlrepro:cqlrepro" "td3bc:td3bc" "bcq:bcq" "dcql:dcql"; do
  IFS=: read args name <<< "$spec"
  timeout -k 10 300 python bench.py --algo $args --cpu-seconds 10 > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  tail -1 $O/bench_$name.json | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 200000 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R && python tools/prof_by_shape.py $O/prof/run_kernel_trace.csv 520 > $O/prof_breakdown.txt && python tools/prof_timeline.py $O/prof/run_kernel_trace.csv > $O/cql_timeline.txt && rm -f $O/prof/run_kernel_trace.csv
tail -14 $O/cql_timeline.txt
