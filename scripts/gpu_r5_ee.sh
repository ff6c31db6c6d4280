# round 5 (ee): whole GPU test suite + smoke() on the final code
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r5_ee_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_ee_smoke.log 2>&1
echo "rc=$?"
tail -1 gpurun_out/r5_ee_tests.log; tail -2 gpurun_out/r5_ee_smoke.log
