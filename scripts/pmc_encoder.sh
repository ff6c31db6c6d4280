#!/bin/bash
# PMC counters of the encoder kernels (run on the GPU box): wave-state breakdown + LDS conflicts.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_enc
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 scripts/encoder_bench.py > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC -d $OUT/pmc -o run -- python3 scripts/encoder_bench.py > $OUT/pmc.log 2>&1
