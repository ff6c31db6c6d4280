# round 6 (v): sequence-packing cost inside the exact team recurrence (scripts/reset_probe.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/reset_probe.py 10 > gpurun_out/r6v_reset_probe.txt 2>&1 || exit $?
echo done
