"""Learning curve of the fused learner in the node loop against the scripted default bot (one JSONL row per
evaluation; see dotaclient_amd/learner/curve.py).

    python scripts/learning_curve.py --budget 600 --eval-every 30 --out profiles/r4_learning_curve.jsonl
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--budget', type=float, default=150.0, help='seconds of training (evaluations excluded)')
    ap.add_argument('--eval-every', type=float, default=25.0)
    ap.add_argument('--eval-games', type=int, default=128)
    ap.add_argument('--model', default='lstm512')
    ap.add_argument('--precision', default='fp32-exact')
    ap.add_argument('--backend', default='auto')
    ap.add_argument('--games', type=int, default=1024)
    ap.add_argument('--threads', type=int, default=12)
    ap.add_argument('--seq-len', type=int, default=1400)
    ap.add_argument('--batch-size', type=int, default=8)
    ap.add_argument('--seq-per-epoch', type=int, default=16)
    ap.add_argument('--lr', type=float, default=1e-4)
    ap.add_argument('--entropy-coef', type=float, default=0.01)
    ap.add_argument('--max-dota-time', type=float, default=600.0)
    ap.add_argument('--pack', type=int, default=1)
    ap.add_argument('--seed', type=int, default=7)
    ap.add_argument('--out', default='gpurun_out/learning_curve.jsonl')
    ap.add_argument('--save-model', default=None, help='write the final weights here (state_dict file)')
    ap.add_argument('--eval-precision', default='fp32', choices=['fp32', 'bf16', 'fp8'])
    ap.add_argument('--mode', default='1v1', choices=['1v1', '5v5'])
    ap.add_argument('--league', default=None, choices=[None, 'pfsp', 'uniform'],
                    help='self-play league opponents (BASELINE config 5)')
    ap.add_argument('--latest-weights-prob', type=float, default=0.8)
    ap.add_argument('--actor-precision', default='bf16', choices=['fp32', 'bf16', 'fp8'])
    ap.add_argument('--replay-gb', type=float, default=0.0, help='on-HBM replay the learner samples from')
    ap.add_argument('--replay-recent', type=int, default=0,
                    help='sample the replay\'s newest N sequences only (0 = the whole buffer)')
    ap.add_argument('--device', default='cuda')
    ap.add_argument('--snapshot-lags', default='120,300,600',
                    help='seconds of training: every row also plays the weights from that long ago (comma list, '
                         'empty = off)')
    ap.add_argument('--snapshot-games', type=int, default=64)
    ap.add_argument('--old-logp', default='actor', choices=['learner', 'actor'])
    ap.add_argument('--advantages', default='vtrace-step', choices=['vtrace-step', 'vtrace-iteration', 'gae'])
    ap.add_argument('--weight-lag', type=int, default=0,
                    help='hold every published version back from the actors until this many newer ones exist '
                         '(staleness on demand: weight age ≈ lag + the loop\'s own)')
    ap.add_argument('--league-matrix', type=int, default=0,
                    help='after the curve: pairwise win rates of this many snapshots spread over the run')
    ap.add_argument('--log-dir', default=None,
                    help='checkpoint directory: resume the curve from it (model, Adam, normalisers, counters) and '
                         'append to --out; --budget is the total over all resumed jobs')
    a = ap.parse_args(argv)
    from dotaclient_amd.learner.curve import run_learning_curve
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, 'a' if a.log_dir else 'w') as fh:
        def emit(row):
            print(json.dumps(row), flush=True)
            fh.write(json.dumps(row) + '\n')
            fh.flush()
        run_learning_curve(budget=a.budget, eval_every=a.eval_every, eval_games=a.eval_games, model=a.model,
                           precision=a.precision, backend=a.backend, games=a.games, threads=a.threads,
                           seq_len=a.seq_len, batch_size=a.batch_size, seq_per_epoch=a.seq_per_epoch, lr=a.lr,
                           entropy_coef=a.entropy_coef, max_dota_time=a.max_dota_time, pack=bool(a.pack),
                           seed=a.seed, device=a.device, on_row=emit, save_model=a.save_model,
                           eval_precision=a.eval_precision, mode=a.mode,
                           log_dir=a.log_dir, league=a.league, latest_weights_prob=a.latest_weights_prob,
                           actor_precision=a.actor_precision, replay_gb=a.replay_gb,
                           snapshot_lags=tuple(float(x) for x in a.snapshot_lags.split(',') if x.strip()),
                           snapshot_games=a.snapshot_games, old_logp=a.old_logp, advantages=a.advantages,
                           weight_lag=a.weight_lag, replay_recent=a.replay_recent,
                           league_matrix_n=a.league_matrix)


if __name__ == '__main__':
    main()
