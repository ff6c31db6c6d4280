# round 5 (aa): 5v5 bf16x3 step with two 64 KB gemm_tn workgroups per CU on the long-K weight gradients
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 20 --model-5v5-exact-extra 10 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_aa.json 2> gpurun_out/r5_aa.err
echo "rc=$?"
