# PMC counters of the fused dX kernel alone (one pass per counter group), on the GPU box
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_dx
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run -- python3 scripts/dx_bench.py fused > $OUT/sq.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_BUSY_CYCLES -d $OUT/sq2 -o run -- python3 scripts/dx_bench.py fused > $OUT/sq2.log 2>&1 && \
for p in sq sq2; do python3 scripts/pmc_summary.py $OUT/$p/run_results.db > $OUT/$p.txt; rm -rf $OUT/$p; done
