# round 5 (final): GPU test suite, full default bench, config 5 at a 200 GB replay, headline + 5v5 step profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5_final_gpu_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r5_bench_final.json 2> gpurun_out/r5_bench_final.err || exit $?
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 20 --league-replay-gb 200 --e2e-5v5-extra 0 > gpurun_out/r5_league_200gb.json 2> gpurun_out/r5_league_200gb.err || exit $?
bash scripts/prof_exact.sh r5_final_exact || exit $?
bash scripts/prof_5v5.sh && mv gpurun_out/prof5_summary.md gpurun_out/r5_final_5v5_bf16x3_summary.md && mv gpurun_out/prof5_timeline.txt gpurun_out/r5_final_5v5_bf16x3_timeline.txt
echo "final rc=$?"
