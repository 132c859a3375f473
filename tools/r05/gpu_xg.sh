#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5xg
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_bcq_parity.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u bench.py --algo bcq --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bcq', d['value'], d['ms_per_step'])"
