# round 6 (k): final GPU suite + smoke on the round's code
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6k_smoke.log 2>&1 || exit $?
timeout -k 10 1050 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r6k_gpu_tests.log 2>&1
echo "pytest rc=$?"
