#!/bin/bash
# round 6: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of every bench
# line's dominant kernel, each file recording the bench description it
# measured (bench.py reads it only for that line), + the SQ pass of the K2 forward
# usage: gpu_pmc6.sh "algo:substr[:suffix[:precision]] ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6pmc
mkdir -p $O
export TMPDIR=/tmp
SPECS=${1:-"cql:q2x6_fwd:_x6 cqldp:q2x6_fwd:_x6 dcql:iqn_head_bwd_rc:_x6 bcq:mlp_x6_wide:_x6 td3bc:gemm_rd_kernel<1, cqlrepro:mlp_x6_wide:_x6 cql:q2x6_fwd:_bf16:bf16"}
for spec in $SPECS; do
  IFS=: read a k sfx prec <<< "$spec"
  PX=""; [ -n "$prec" ] && PX="--precision $prec"
  cd /tmp
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/${a}${sfx}_f -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $a $PX --transitions 100000 --desc-out $O/${a}${sfx}_desc.json > $O/${a}${sfx}_f.log 2>&1 || { tail -5 $O/${a}${sfx}_f.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/${a}${sfx}_w -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo $a $PX --transitions 100000 > $O/${a}${sfx}_w.log 2>&1 || { tail -5 $O/${a}${sfx}_w.log; exit 1; }
  cd $R && python tools/pmc_summarize.py $O/${a}${sfx}_f $O/${a}${sfx}_w $k $O/r06_pmc_traffic_${a}${sfx}.json $O/${a}${sfx}_desc.json 6 | cut -c1-400
  find $O -name "*counter_collection.csv" -size +20M -delete
done
if [ -n "$SQ" ]; then
  cd /tmp
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/sq_fwd -o run --output-format csv -- python3 $R/tools/pmc_dominant.py --algo cql --transitions 100000 > $O/sq_fwd.log 2>&1 || { tail -5 $O/sq_fwd.log; exit 1; }
  cd $R && python tools/pmc_sq_summary.py $O/sq_fwd q2x6_fwd > $O/r06_pmc_sq_k2_fwd.txt; cat $O/r06_pmc_sq_k2_fwd.txt
  find $O -name "*counter_collection.csv" -size +20M -delete
fi
