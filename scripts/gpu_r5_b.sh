# round 5 (b): actor core tests, then the half-team exact tests and the learner step at half 0/1 × 1/2/4 chunks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_actor_gpu.py tests/test_actor_fp8.py -m gpu > gpurun_out/r5_actor_tests.log 2>&1
rc=$?
echo "actor tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DCA_TEAM_HALF=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_exact_mode.py -m gpu > gpurun_out/r5_half_exact_tests.log 2>&1
rc=$?
echo "half exact tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/r5_half_sweep.txt
for h in 0 1; do for c in 1 2 4; do
  DCA_TEAM_HALF=$h DCA_PIPELINE_CHUNKS=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_half_h${h}_c${c}.json 2> gpurun_out/r5_half_h${h}_c${c}.err || exit $?
  echo "half=$h chunks=$c $(python -c "import json;d=json.load(open('gpurun_out/r5_half_h${h}_c${c}.json'));print(d['ms_per_step'])")" >> gpurun_out/r5_half_sweep.txt
done; done
