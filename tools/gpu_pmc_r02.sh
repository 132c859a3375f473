# r02 PMC: SQ pass over the eager K2 step + FETCH/WRITE passes of the dominant kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq_step -o run --output-format csv -- python3 $R/tools/pmc_step.py > $R/gpurun_out/pmc_sq_step.log 2>&1 || exit $?
cd $R && python tools/pmc_reconcile.py gpurun_out/pmc_sq_step gpurun_out/r02_pmc_sq_cql.txt || exit $?
bash tools/pmc_pass.sh cql mlp_fwd_kernel || exit $?
cd $R && find gpurun_out/pmc_sq_step gpurun_out/pmc_fetch_cql gpurun_out/pmc_write_cql -name "*.csv" -size +20M -delete
