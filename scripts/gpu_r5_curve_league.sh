# round 5: BASELINE config 5 as a learning curve — PFSP self-play league, fp8 actor policy step, every minibatch from
# a 100 GB on-HBM replay; validation against the default bot with the IEEE-fp32 actor; 8 min of training
# (DCA_TEAM_PATIENT=1: a first try at the 2 s hand-off deadline failed within a minute, persistent kernel error code 2 —
# the config-5 stalls of profiles/r5_replay_timeout.md, here with the actor in the learner process)
set -o pipefail
mkdir -p gpurun_out
DCA_TEAM_PATIENT=1 timeout -k 10 1000 python -u scripts/learning_curve.py --budget 480 --eval-every 60 --eval-games 256 \
  --league pfsp --latest-weights-prob 0.8 --actor-precision fp8 --replay-gb 100 \
  --out gpurun_out/r5_curve_league.jsonl > gpurun_out/r5_curve_league.log 2>&1
echo "curve rc=$?"
