# round 5 (pp): config 5 at a 200 GB replay at the 2 s hand-off deadline after the actor-priority fix, then the whole
# GPU test suite and smoke() on the final code
set -o pipefail
mkdir -p gpurun_out
DCA_TEAM_PATIENT=0 timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 20 --league-replay-gb 200 --e2e-5v5-extra 0 > gpurun_out/r5_pp_200.json 2> gpurun_out/r5_pp_200.err && \
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r5_pp_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_pp_smoke.log 2>&1
echo "rc=$?"
tail -1 gpurun_out/r5_pp_tests.log; tail -1 gpurun_out/r5_pp_smoke.log
