# half-team (16 CU-exclusive workgroups per XCD team) probe: standalone recurrence alone / beside a side GEMM,
# outputs vs the 32-workgroup teams, the exact parity tests under half teams, and the learner step at 1 / 2 / 4 chunks
set -o pipefail
mkdir -p gpurun_out
DCA_TEAM_HALF=0 timeout -k 10 120 python -u scripts/team_half_probe.py /tmp/half0.pt > gpurun_out/r5_half_probe.txt 2>&1 || exit $?
DCA_TEAM_HALF=1 timeout -k 10 120 python -u scripts/team_half_probe.py /tmp/half1.pt /tmp/half0.pt >> gpurun_out/r5_half_probe.txt 2>&1 || exit $?
DCA_TEAM_HALF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_exact_mode.py -m gpu > gpurun_out/r5_half_exact_tests.log 2>&1 || exit $?
for h in 0 1; do for c in 1 2 4; do
  DCA_TEAM_HALF=$h DCA_PIPELINE_CHUNKS=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_half_h${h}_c${c}.json 2> gpurun_out/r5_half_h${h}_c${c}.err || exit $?
  echo "half=$h chunks=$c $(python -c "import json;d=json.load(open('gpurun_out/r5_half_h${h}_c${c}.json'));print(d['ms_per_step'])")" >> gpurun_out/r5_half_probe.txt
done; done
