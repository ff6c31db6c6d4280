# 5v5 step profile + node-loop A/B of the actor policy precision
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/prof_5v5.sh && \
timeout -k 10 400 python -u scripts/e2e_ab.py 15 2048,12,bf16 2048,12,fp8 2048,14,fp8 > gpurun_out/e2e_ab.log 2> gpurun_out/e2e_ab.err
