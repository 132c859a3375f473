# r04 iteration 18: the SAC actor head in the policy trunk backward's prologue
# (d3a_q2_bwd_actor_head): A/B bitwise test, CQL / SAC suites, K2 bench A/B + timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_cql_parity.py -k "actor_head_in_trunk or hopper or k4" > gpurun_out/i18_cql.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_sac_parity.py tests/test_gpu_dp.py tests/test_gpu_q2_bwd.py tests/test_gpu_production_path.py tests/test_gpu_capture_gc.py tests/test_gpu_api.py tests/test_gpu_actor_q.py > gpurun_out/i18_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0 1; do D3A_HEAD_IN_TRUNK=$x timeout -k 10 300 python bench.py --algo cql --steps 2000 --warmup 50 --no-cpu-baseline | sed "s/^/head_in_trunk $x: /" >> gpurun_out/i18_bench.txt 2>/dev/null || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_cql18 -o run --output-format csv -- python3 $R/bench.py --algo cql --steps 200 --warmup 20 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_cql18.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_cql18/run_kernel_trace.csv > gpurun_out/tl_cql18.txt; rm -f gpurun_out/tl_cql18/run_kernel_trace.csv
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/i19_conv.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_BWD_X6=$x timeout -k 10 120 python tools/bench_conv_bwd.py >> gpurun_out/i19_convbench.jsonl 2>gpurun_out/i19_convbench.err || exit $?; done
D3A_CONV_BWD_X6=0 SPLITS=32 timeout -k 10 120 python tools/bench_conv_bwd.py >> gpurun_out/i19_convbench.jsonl 2>>gpurun_out/i19_convbench.err || exit $?
timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_discrete_cql.py tests/test_gpu_arbiters.py tests/test_gpu_dqn.py tests/test_gpu_sbf16.py tests/test_gpu_sampler.py > gpurun_out/i19_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_BWD_X6=$x D3A_CONV_BWD_X=$x timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/conv_bwd_x6+x $x: /" >> gpurun_out/i19_bench.txt 2>/dev/null || exit $?; done
D3A_FC_SPLITK=0 timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/fc_splitk 0 only: /" >> gpurun_out/i19_bench.txt 2>/dev/null || exit $?
D3A_CONV_BWD_X=0 timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/conv_bwd_x 0 only: /" >> gpurun_out/i19_bench.txt 2>/dev/null || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_dcql19 -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 60 --warmup 10 --no-cpu-baseline --transitions 100000 > $R/gpurun_out/tl_dcql19.log 2>&1 || exit $?
python tools/prof_timeline.py gpurun_out/tl_dcql19/run_kernel_trace.csv > gpurun_out/tl_dcql19.txt; rm -f gpurun_out/tl_dcql19/run_kernel_trace.csv
