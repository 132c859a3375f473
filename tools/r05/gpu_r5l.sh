#!/bin/bash
# round 5: defaults after the branch / deep-x6 A/Bs -- benches of every line,
# then the PMC passes (tools/r05/gpu_pmc5.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5l
cd $R && mkdir -p $O
B="timeout -k 10 200 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline --transitions 100000"
for a in cql cqlrepro bcq dcql td3bc; do
  $B --algo $a > $O/b_$a.json 2>$O/b_$a.err || exit 1; echo $a; cut -c1-200 $O/b_$a.json
done
bash tools/r05/gpu_pmc5.sh
