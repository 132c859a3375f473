#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5p32
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "parts or small_mlp" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_bcq.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/prof_bcq/run_kernel_trace.csv > $O/tl_bcq.txt && rm -f $O/prof_bcq/run_kernel_trace.csv && head -14 $O/tl_bcq.txt && tail -1 $O/tl_bcq.txt
