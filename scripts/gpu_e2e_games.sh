# node-loop game count A/B (games per actor process; 2 players per game)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/e2e_ab.py 15 4096,14,bf16,1 3072,14,bf16,1 2048,14,bf16,1 3072,14,bf16,1 > gpurun_out/e2e_games2.log 2> gpurun_out/e2e_games2.err
