# round 5 (u): is the node loop CPU-quota throttled? cgroup cpu.stat around e2e runs with 14 / 11 actor threads
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 15 --league-replay-extra 0 --e2e-5v5-extra 0"
S=gpurun_out/r5_u_cpustat.txt
{ cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/cgroup; echo "--- before"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null; } > $S
DCA_STAGE_PROF=1 timeout -k 10 240 python -u bench.py $B --e2e-threads 14 > gpurun_out/r5_u_14.json 2> gpurun_out/r5_u_14.err && \
{ echo "--- after 14"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null; } >> $S && \
DCA_STAGE_PROF=1 timeout -k 10 240 python -u bench.py $B --e2e-threads 11 > gpurun_out/r5_u_11.json 2> gpurun_out/r5_u_11.err && \
{ echo "--- after 11"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null; } >> $S
echo "rc=$?"
