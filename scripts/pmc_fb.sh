#!/bin/bash
# Counter passes over the fused fp32 encoder backward (scripts/enc_fb_probe.py); results under gpurun_out/fbpmc*
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/fbpmc1 -o run -- python scripts/enc_fb_probe.py 2 > gpurun_out/fbpmc.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/fbpmc2 -o run -- python scripts/enc_fb_probe.py 2 >> gpurun_out/fbpmc.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d gpurun_out/fbpmc3 -o run -- python scripts/enc_fb_probe.py 2 >> gpurun_out/fbpmc.log 2>&1
