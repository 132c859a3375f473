#!/bin/bash
# BCQ launch folds (the parts-path row write-out, the in-launch target):
# tests, a K3 line and its step timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5q
cd $R && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_bcq_parity.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --algo bcq --steps 2000 --warmup 50 --no-cpu-baseline > $O/bcq.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bcq.json').read().strip().splitlines()[-1]); print('bcq', d['value'], d['ms_per_step'])"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_bcq.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/prof_bcq/run_kernel_trace.csv > $O/tl_bcq.txt && rm -f $O/prof_bcq/run_kernel_trace.csv && tail -1 $O/tl_bcq.txt
