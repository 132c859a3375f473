#!/bin/bash
# the small forward's MFMA head: its tests, BCQ parity, K3 bench A/B + timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5sw
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bcq_parity.py tests/test_gpu_mlp_bwd_small.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1; do
  D3A_SMALL_WIDE=$v timeout -k 10 200 python -u bench.py --algo bcq --steps 1000 --warmup 50 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('small_wide=$v', d['value'], d['ms_per_step'])"
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bcq -o run --output-format csv -- python3 $R/bench.py --algo bcq --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_bcq.log 2>&1 || exit 1
cd $R && python tools/prof_timeline.py $O/prof_bcq/run_kernel_trace.csv > $O/tl_bcq.txt && rm -f $O/prof_bcq/run_kernel_trace.csv && grep "small\|step:" $O/tl_bcq.txt
