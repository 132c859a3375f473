#!/bin/bash
# K2 split-bf16 forward: the round-5 schedule (default), without the tile-major
# last chunk (D3A_X6_PROBE=128) and
# round-4 schedule (D3A_X6_PROBE=64), timing and stamps, then the x6 / CQL tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g
cd $R && mkdir -p $O
for v in 0 128 64 0 128 64; do
  D3A_X6_PROBE=$v timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --reps 1000 >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
done
D3A_X6_PROBE=16 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
D3A_X6_PROBE=144 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
cut -c1-420 $O/fwd.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_x6t.py tests/test_gpu_cql_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
