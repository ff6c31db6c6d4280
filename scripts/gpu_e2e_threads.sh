# node loop: actor host threads A/B after the host-loop fixes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/e2e_ab.py 15 2048,12,bf16 2048,14,bf16 1024,12,bf16 > gpurun_out/e2e_ab4.log 2> gpurun_out/e2e_ab4.err
