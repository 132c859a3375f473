#!/bin/bash
# a test subset, then the K2 kernel timeline and a 2000-step bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6t_$1
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread $2 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ALGO=${3:-cql} timeout -k 10 400 bash tools/profiling/gpu_timeline.sh || exit 1
tail -14 gpurun_out/tl_${3:-cql}.txt
timeout -k 10 300 python -u bench.py --algo ${3:-cql} --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
