# BASELINE config 4 end to end: the node loop on the 5v5 model (bench extra e2e_5v5 alone)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 15 > gpurun_out/e2e5.log 2> gpurun_out/e2e5.err
