# PMC counters of the IEEE-fp32 learner kernels (standalone, scripts/exact_kernels_bench.py): MFMA busy, wave states,
# LDS conflicts — one counter pass per run (results under gpurun_out/pmc_exact/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_exact
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $OUT/p1 -o run -- python3 scripts/exact_kernels_bench.py 3 > $OUT/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $OUT/p2 -o run -- python3 scripts/exact_kernels_bench.py 3 > $OUT/p2.log 2>&1 && \
python3 scripts/pmc_summary.py $OUT/p1/run_results.db x_kernel gemm_tn_exact dpre_dx > $OUT/summary.txt && \
python3 scripts/pmc_summary.py $OUT/p2/run_results.db x_kernel gemm_tn_exact dpre_dx >> $OUT/summary.txt && rm -rf $OUT/p1 $OUT/p2
