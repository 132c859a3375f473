#!/bin/bash
# round 6: SQ counters of the reproduction config's weight-gradient GEMM
# (gemm_sbf16_kernel<6, true, true>, 8 K tiles a split) over a short bench run:
# MFMA / VALU issue, wave waits, LDS bank conflicts -> r06_pmc_sq_repro_dw*.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6pmc_sb
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/sq1 -o run --output-format csv -- python3 $R/bench.py --algo cqlrepro --steps 10 --warmup 3 --no-cpu-baseline --transitions 100000 > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
cd $R && python tools/pmc_sq_summary.py $O/sq1 gemm_sbf16 > $O/r06_pmc_sq_repro_dw.txt; cat $O/r06_pmc_sq_repro_dw.txt
find $O -name "*counter_collection.csv" -size +20M -delete
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL -d $O/sq2 -o run --output-format csv -- python3 $R/bench.py --algo cqlrepro --steps 10 --warmup 3 --no-cpu-baseline --transitions 100000 > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
cd $R && python tools/pmc_sq_summary.py $O/sq2 gemm_sbf16 > $O/r06_pmc_sq_repro_dw_lds.txt; cat $O/r06_pmc_sq_repro_dw_lds.txt
find $O -name "*counter_collection.csv" -size +20M -delete
