# r04 measurement 1: per-launch timelines (K2 x6 / fp32, bf16 line, K3 x6), PMC
# traffic of the x6 dominant kernel, SQ counters of the x6 forward / backward,
# short-window bench sensitivity (warm-up / step count), x1 kernel test
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -s tests/test_gpu_bf16.py > gpurun_out/p1_bf16_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
export TMPDIR=/tmp
for cfg in "cql x6 fp32" "cql fp32 fp32" "cql x6 bf16" "bcq x6 fp32"; do
  set -- $cfg
  tag=$1_$2_$3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tl_$tag -o run --output-format csv -- python3 $R/bench.py --algo $1 --critic-gemm $2 --precision $3 --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > $R/gpurun_out/tl_$tag.log 2>&1 || exit $?
  python tools/prof_timeline.py gpurun_out/tl_$tag/run_kernel_trace.csv > gpurun_out/tl_$tag.txt && python tools/prof_by_shape.py gpurun_out/tl_$tag/run_kernel_trace.csv 320 > gpurun_out/tl_${tag}_shape.txt || exit $?
  rm -f gpurun_out/tl_$tag/run_kernel_trace.csv
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_x6 -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cql --critic-gemm x6 > $R/gpurun_out/pmc_fetch_x6.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_x6 -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cql --critic-gemm x6 > $R/gpurun_out/pmc_write_x6.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_bf16 -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cql --precision bf16 > $R/gpurun_out/pmc_fetch_bf16.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_bf16 -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cql --precision bf16 > $R/gpurun_out/pmc_write_bf16.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq_fwd_x6 -o run --output-format csv -- python3 $R/tools/bench_fwd.py --x6 --reps 20 > $R/gpurun_out/pmc_sq_fwd_x6.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq_bwd_x6 -o run --output-format csv -- python3 $R/tools/bench_q2.py --x6 --reps 20 > $R/gpurun_out/pmc_sq_bwd_x6.log 2>&1 || exit $?
cd $R
python tools/pmc_summarize.py gpurun_out/pmc_fetch_x6 gpurun_out/pmc_write_x6 q2x6_fwd gpurun_out/r04_pmc_traffic_cql_x6.json > gpurun_out/pmc_sum_x6.log 2>&1
python tools/pmc_summarize.py gpurun_out/pmc_fetch_bf16 gpurun_out/pmc_write_bf16 q2x6_fwd gpurun_out/r04_pmc_traffic_cql_bf16.json > gpurun_out/pmc_sum_bf16.log 2>&1
for sw in "20 5" "20 50" "100 5" "2000 50"; do set -- $sw; timeout -k 10 200 python bench.py --critic-gemm x6 --steps $1 --warmup $2 --no-cpu-baseline >> gpurun_out/p1_window.jsonl 2>/dev/null || exit $?; done
