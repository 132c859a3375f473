#!/bin/bash
# A/B in one call: the tree against ab_old/ (the same tree built with the
# per-value split of commit 4e114bc), K5 and K2 lines alternately
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5ab
mkdir -p $O
: > $O/ab.jsonl
for round in 1 2; do
  for side in new old; do
    D=$R; [ $side = old ] && D=$R/ab_old
    for a in dcql cql; do
      (cd $D && timeout -k 10 300 python -u bench.py --algo $a --steps 500 --warmup 50 --no-cpu-baseline --transitions 200000) > $O/one.json 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
      python -c "
import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print('$side', '$a', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
    done
  done
done
