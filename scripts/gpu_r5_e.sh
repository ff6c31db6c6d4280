# round 5 (e): exact 5v5 — attention block kernel tests (bf16x3 + exact twins), exact encoder bwd with given ∂E0,
# 5v5 exact step vs fp64, the bf16x3 5v5 fp64 test, then the 5v5 timings (bf16x3 / exact) and a timeline of each
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_attn_kernels.py "tests/test_exact_mode.py::test_exact_5v5_step_matches_fp64" "tests/test_fp32_kernels.py::test_fused_fp32_presets_match_fp64[5v5-ppo]" -m gpu > gpurun_out/r5_5v5x_tests.log 2>&1
rc=$?
echo "5v5 exact tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --model 5v5 --steps 10 --warmup 3 --bf16x3-extra 1 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_5v5x_bench.json 2> gpurun_out/r5_5v5x_bench.err || exit $?
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof5x -o run -- python3 $R/bench.py --model 5v5 --precision fp32-exact --steps 5 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0 > $R/gpurun_out/prof5x.log 2>&1 || exit $?
cd $R && python scripts/prof_summary.py gpurun_out/prof5x/run_results.db --steps 9 > gpurun_out/r5_5v5_exact_summary.md && python scripts/step_timeline.py gpurun_out/prof5x/run_results.db > gpurun_out/r5_5v5_exact_timeline.txt && rm -rf gpurun_out/prof5x
