set -o pipefail
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model 5v5 --steps 3 --warmup 2 --actor 0 > $GRAFT_REPO_ROOT/gpurun_out/prof5.log 2>&1
