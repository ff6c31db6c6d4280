# actor runtime threads (standalone) and node-loop game count sweeps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--steps 3 --warmup 2 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
for t in 14 16 14 16; do
  timeout -k 10 300 python -u bench.py $B --actor-threads $t > gpurun_out/at_$t.log 2>&1 || exit $?
  python - $t >> gpurun_out/at_summary.txt <<'PY'
import json, sys
l = [x for x in open(f'gpurun_out/at_{sys.argv[1]}.log') if x.startswith('{')][-1]
a = json.loads(l)['actor']
print('threads', sys.argv[1], round(a['steps_per_s']), round(a['protobuf_runtime_steps_per_s']))
PY
done
timeout -k 10 300 python -u scripts/e2e_ab.py 15 3072,14,bf16,1 2048,14,bf16,1 > gpurun_out/e2e_games.log 2> gpurun_out/e2e_games.err
