#!/bin/bash
# Pre-split weight images: kernel tests, forward A/B, CQL parity, K2 A/B bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6a
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_presplit.py tests/test_gpu_x6.py > $O/tests1.log 2>&1 || { tail -40 $O/tests1.log; exit 1; }
tail -2 $O/tests1.log
for v in 0 1 0 1 0 1; do
  P=""; [ $v = 1 ] && P="--pre"
  timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --reps 2000 --warm 1000 $P >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
done
cut -c1-300 $O/fwd.jsonl
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py tests/test_gpu_sac_parity.py tests/test_gpu_cql_softmax.py tests/test_torch_ops.py > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -2 $O/tests2.log
for v in 1 0 1 0; do :
  D3A_X6_PRESPLIT=$v timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('presplit=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
for v in 1 0 1 0; do
  D3A_OP_REPLAY=$v timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_op$v.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_op$v.json').read().strip().splitlines()[-1]); print('op_replay=$v', d['value'], d['ms_per_step'], d['host']['host_us_per_step'])"
done
