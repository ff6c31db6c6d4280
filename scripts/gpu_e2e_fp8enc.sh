# node loop on the fp8 actor step: wave-parallel vs per-unit entity encoder (co-residency beside the recurrence)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DCA_FP8_ENC_PER_UNIT=0 timeout -k 10 200 python -u scripts/e2e_ab.py 15 2048,14,fp8,1 > gpurun_out/e2e_fp8w.log 2> gpurun_out/e2e_fp8w.err && \
DCA_FP8_ENC_PER_UNIT=1 timeout -k 10 200 python -u scripts/e2e_ab.py 15 2048,14,fp8,1 > gpurun_out/e2e_fp8u.log 2> gpurun_out/e2e_fp8u.err && \
DCA_FP8_ENC_PER_UNIT=0 timeout -k 10 200 python -u scripts/e2e_ab.py 15 2048,14,fp8,1 > gpurun_out/e2e_fp8w2.log 2> gpurun_out/e2e_fp8w2.err
