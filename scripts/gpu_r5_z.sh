# round 5 (z): config 5 at a 200 GB replay failed the 2 s recurrence hand-off timeout within 5 s of the loop
# (r5_league_200gb): same run with the patient (60 s) timeout — does it complete, and how long is the worst step?
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 20 --e2e-5v5-extra 0"
{ rocm-smi --showmeminfo vram 2>&1 | grep -i "total" ; } > gpurun_out/r5_z_mem.txt || true
DCA_TEAM_PATIENT=1 timeout -k 10 400 python -u bench.py $B --league-replay-gb 200 > gpurun_out/r5_z_200p.json 2> gpurun_out/r5_z_200p.err && \
timeout -k 10 400 python -u bench.py $B --league-replay-gb 150 > gpurun_out/r5_z_150.json 2> gpurun_out/r5_z_150.err
echo "rc=$?"
