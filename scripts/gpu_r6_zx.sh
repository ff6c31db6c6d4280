# round 6 (zx): same-box A/B of the backward's reset-flag form: compare at load (current build) vs deferred (_C_def.so)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 200 python -u scripts/reset_probe.py 20 > gpurun_out/r6zx_cur_$i.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/reset_probe.py 20 scripts/_C_def.so > gpurun_out/r6zx_def_$i.txt 2>&1 || exit $?
done
echo done
