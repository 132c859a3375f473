#!/bin/bash
# round 6, K5 Adam: DiscreteCQL GPU tests, a step timeline, and the adam_kernel's
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes over a short bench, adam only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/k5
mkdir -p $O
export TMPDIR=/tmp
cd $R && timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_discrete_cql.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ALGO=dcql timeout -k 10 320 bash tools/profiling/gpu_timeline.sh || exit 1
cp gpurun_out/tl_dcql.txt gpurun_out/tl_dcql.log $O/
grep -E "adam|steps/s|value" $O/tl_dcql.txt | head; tail -1 $O/tl_dcql.log | cut -c1-300
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex adam_kernel -d $O/$c -o run --output-format csv -- python3 $R/bench.py --algo dcql --steps 10 --warmup 3 --no-cpu-baseline --transitions 100000 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
cd $R && python tools/k5_adam_pmc.py $O/FETCH_SIZE $O/WRITE_SIZE | tee $O/adam_pmc.txt
find $O -name "*counter_collection.csv" -size +20M -delete
