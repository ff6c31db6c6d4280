# round 6 (zw): backward reset flags from an LDS bit image — packing/exact GPU tests, then a same-box A/B of the
# reset probe: original build (scripts/_C_orig.so) vs the current one
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_packing.py tests/test_exact_mode.py > gpurun_out/r6zw_tests.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 200 python -u scripts/reset_probe.py 20 scripts/_C_orig.so > gpurun_out/r6zw_orig_$i.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/reset_probe.py 20 > gpurun_out/r6zw_new_$i.txt 2>&1 || exit $?
done
echo done
