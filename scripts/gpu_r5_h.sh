# round 5 (h): determinism of the fused step, the learner-async tests, the exact 5v5 test after the colsum change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/determinism_check.py > gpurun_out/r5_determinism.txt 2>&1
echo "determinism rc=$?"
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_learner_async.py "tests/test_exact_mode.py::test_exact_5v5_step_matches_fp64" "tests/test_exact_mode.py::test_exact_fused_step_deploy_shape_matches_fp64" -m gpu > gpurun_out/r5_h_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u scripts/diag_5v5_head.py 1400 > gpurun_out/r5_diag_5v5_head.txt 2>&1
echo "diag rc=$?"
