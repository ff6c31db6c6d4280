# round 6 (t): what overlaps the learner's recurrence in the node loop (feeder vs actor), scripts/e2e_overlap.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
E="--steps 3 --warmup 1 --bf16x3-extra 0 --vtrace-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 8 --e2e-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0"
rm -rf /tmp/prof_feed /tmp/prof_act
DCA_E2E_FEEDER=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_feed -- python3 bench.py $E > gpurun_out/r6t_feed.json 2> gpurun_out/r6t_feed.err || exit $?
python3 scripts/e2e_overlap.py /tmp/prof_feed > gpurun_out/r6_e2e_overlap_feeder.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_act -- python3 bench.py $E > gpurun_out/r6t_act.json 2> gpurun_out/r6t_act.err || exit $?
python3 scripts/e2e_overlap.py /tmp/prof_act > gpurun_out/r6_e2e_overlap_actor.txt 2>&1 || exit $?
echo done
