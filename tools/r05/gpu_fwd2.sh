#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5e
cd $R && mkdir -p $O
for v in 0 32 8 0; do
  D3A_X6_PROBE=$v timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --reps 1000 >> $O/fwd_probe.jsonl 2>>$O/fwd_probe.err || exit $?
done
D3A_X6_PROBE=16 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 >> $O/fwd_probe.jsonl 2>>$O/fwd_probe.err || exit $?
cat $O/fwd_probe.jsonl | cut -c1-400
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_x6t.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
