# round 5 (o): kernel trace of the node loop (learner + actor process on one GPU) -> learner idle gaps / overlap
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rm -rf /tmp/prof_e2e && rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_e2e -- python3 bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 8 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_prof_e2e.json 2> gpurun_out/r5_prof_e2e.err
echo "prof rc=$?"
python3 scripts/e2e_gaps.py /tmp/prof_e2e --window-s 5 > gpurun_out/r5_e2e_gaps2.txt 2>&1
echo "gaps rc=$?"
ls -la /tmp/prof_e2e/* | head -20 >> gpurun_out/r5_e2e_gaps2.txt
