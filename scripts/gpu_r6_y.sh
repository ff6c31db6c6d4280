# round 6 (y): recurrence per-call time, learner alone vs node loop with the CPU feeder, packed vs padded sequences
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L="--steps 20 --warmup 5 --bf16x3-extra 0 --vtrace-extra 1 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --e2e-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0"
E="--steps 3 --warmup 1 --bf16x3-extra 0 --vtrace-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 8 --e2e-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0"
rm -rf /tmp/prof_l /tmp/prof_p1 /tmp/prof_p0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_l -- python3 bench.py $L > gpurun_out/r6y_learner.json 2> gpurun_out/r6y_learner.err || exit $?
python3 scripts/e2e_overlap.py /tmp/prof_l --window-s 1000 > gpurun_out/r6y_learner.txt 2>&1 || exit $?
DCA_E2E_FEEDER=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_p1 -- python3 bench.py $E --e2e-pack 1 > gpurun_out/r6y_p1.json 2> gpurun_out/r6y_p1.err || exit $?
python3 scripts/e2e_overlap.py /tmp/prof_p1 > gpurun_out/r6y_p1.txt 2>&1 || exit $?
DCA_E2E_FEEDER=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_p0 -- python3 bench.py $E --e2e-pack 0 > gpurun_out/r6y_p0.json 2> gpurun_out/r6y_p0.err || exit $?
python3 scripts/e2e_overlap.py /tmp/prof_p0 > gpurun_out/r6y_p0.txt 2>&1 || exit $?
echo done
