# node loop: one vs two actor processes per rank (games / threads split); plus the exact / bf16x3 step profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/e2e_ab.py 15 2048,14,bf16,1 2048,14,bf16,2 2048,16,bf16,2 > gpurun_out/e2e_ab6.log 2> gpurun_out/e2e_ab6.err && \
bash scripts/prof_exact.sh profx && bash scripts/prof_1v1.sh
