# round 6 (x): same-box A/B of the team recurrence, previous build (scripts/_C_prev.so) vs the current one
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u scripts/reset_probe.py 20 scripts/_C_prev.so > gpurun_out/r6x_prev_$i.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/reset_probe.py 20 > gpurun_out/r6x_new_$i.txt 2>&1 || exit $?
done
echo done
