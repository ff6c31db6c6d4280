#!/bin/bash
# PMC counter passes over the learner step (eager, no hipGraph, so every dispatch is attributed):
# wave/MFMA/LDS counters, L2 fetch bytes, L2 write bytes + hit/miss. One rocprofv3 run per pass
# (counter limits per block: 8 SQ, 4 TCC, 2 GRBM). Run on the GPU box; summarise with scripts/pmc_summary.py.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_step
mkdir -p $OUT
CMD="python3 bench.py --steps 2 --warmup 2 --actor 0 --e2e 0 --e2e-5v5-extra 0 --bf16x3-extra 0 --graph 0"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run -- $CMD > $OUT/sq.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1
for p in sq fetch write; do
    python3 scripts/pmc_summary.py $OUT/$p/run_results.db > $OUT/$p.txt
    rm -rf $OUT/$p
done
grep -v "^[WE]2026\|^W[0-9]\|^E[0-9]" $OUT/sq.log | tail -5 > $OUT/bench_tail.txt || true
rm -f $OUT/counters.txt.full
du -sh $OUT
