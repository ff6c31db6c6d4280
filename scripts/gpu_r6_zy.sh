# round 6 (zy): exact / packing GPU tests and the reset probe after reverting the backward flag change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_packing.py tests/test_exact_mode.py > gpurun_out/r6zy_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/reset_probe.py 20 > gpurun_out/r6zy_reset_probe.txt 2>&1 || exit $?
echo done
