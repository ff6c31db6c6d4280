"""Learning curve of the node loop against the scripted default bot — the reference's only quality signal.

The actor (VecActor, native engine, self-play on the latest weights) feeds an in-process DotaOptimizer (the fused
IEEE-fp32 learner by default, lstm512, the reference deploy shape 8 × 1400); every ``eval_every`` seconds of training
the learner's current weights play ``eval_games`` games against the default bot (actor/validate.py — the reference's
validation agent, /root/reference/agent.py:905-927 / 415-434) and one row is emitted: training wall time, iterations,
learner samples, actor steps, ``game/rewards_sum``, ``game/win_rate`` and the per-key rewards. Evaluation games use a
fixed seed, so every row plays the same opening positions; evaluation time is excluded from ``t_train``.

Beyond the reference (round 6): the default-bot win rate saturates (5v5 ends games in ≈130 steps at 100 % wins), so
every row also plays the current weights head-to-head against frozen snapshots of itself from ``snapshot_lags``
seconds of training earlier (``snap/win_rate_vs_<lag>``, actor/validate.py ``evaluate_vs_snapshot``), and a league
curve logs the training league's score against its pool (``league/score``, ``league/pool``). Every row carries the
learner's ``approx_kl`` / ``clipfrac`` / ``avg_weight_age`` and the off-policy diagnostics of the learner-side
policy_old pass (``offpolicy/*``).

Used by ``scripts/learning_curve.py`` (profiles/r4_learning_curve.jsonl) and tests/test_learning.py.
"""
from __future__ import annotations

import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional


def run_learning_curve(budget: float = 150.0, eval_every: float = 25.0, eval_games: int = 128,
                       model: str = 'lstm512', precision: str = 'fp32-exact', backend: str = 'auto',
                       games: int = 1024, threads: int = 12, seq_len: int = 1400, batch_size: int = 8,
                       seq_per_epoch: int = 16, lr: float = 1e-4, entropy_coef: float = 0.01,
                       max_dota_time: float = 600.0, pack: bool = True, seed: int = 7, device: str = 'cuda',
                       eval_seed: int = 4242, on_row: Optional[Callable[[Dict], None]] = None,
                       save_model: Optional[str] = None, eval_precision: str = 'fp32',
                       mode: str = '1v1', log_dir: Optional[str] = None, league: Optional[str] = None,
                       latest_weights_prob: float = 0.8, actor_precision: str = 'bf16',
                       replay_gb: float = 0.0, snapshot_lags=(120.0, 300.0, 600.0), snapshot_games: int = 64,
                       old_logp: str = 'actor', league_matrix_n: int = 0,
                       advantages: str = 'vtrace-step', weight_lag: int = 0,
                       replay_recent: int = 0) -> List[Dict]:
    """Train for ``budget`` seconds (evaluations excluded) and return the evaluation rows (the first one before
    any training). ``on_row`` is called with every row as it is produced; ``save_model``: path that receives the
    final weights (a reference-format state_dict file). ``eval_precision``: the validation games' policy step.

    ``log_dir``: keep the optimizer's checkpoints there (the latest one only) and resume from them — model, Adam
    state and return normalisers (DotaOptimizer's resume) plus the curve's own counters (``curve_state.json``), so a
    long curve runs as several shorter jobs; ``budget`` is then the total, counted from the first job.

    BASELINE config 5 as a curve: ``league`` ('pfsp' / 'uniform', actor/league.py) makes the actors play the latest
    weights against sampled past versions (``latest_weights_prob`` of the games self-play the latest), the actor's
    policy step runs at ``actor_precision`` ('fp8' for config 5), and ``replay_gb`` > 0 trains every minibatch from
    an on-HBM replay of that size (learner/replay.py) instead of the iteration's fresh rollouts — uniformly over the
    whole buffer, or over its ``replay_recent`` newest sequences."""
    import json
    import os

    import torch
    from ..actor.validate import evaluate_vs_default_bot, evaluate_vs_snapshot
    from ..actor.vec import VecActor
    from ..actor.weights import WeightStore
    from ..transport.broker import InProcBroker
    from .optimizer import DotaOptimizer, OptimizerConfig

    torch.manual_seed(seed)
    tmp = log_dir or tempfile.mkdtemp(prefix='dca_curve_')
    os.makedirs(tmp, exist_ok=True)
    state_path = os.path.join(tmp, 'curve_state.json')
    resumed = {}
    if log_dir and os.path.exists(state_path):
        with open(state_path) as fh:
            resumed = json.load(fh)
    broker = InProcBroker(maxsize=256, drop_oldest=True)
    cfg = OptimizerConfig(log_dir=tmp, epochs=1, seq_per_epoch=seq_per_epoch, batch_size=batch_size,
                          seq_len=seq_len, model=model, precision=precision, device=device, backend=backend,
                          learning_rate=lr, entropy_coef=entropy_coef, checkpoint_keep=1 if log_dir else 2,
                          run_local=True,
                          xp_timeout=300.0, histogram_freq=10 ** 9, async_checkpoint=True, prefetch_rollouts=64,
                          pack_sequences=bool(pack), seed=seed, replay_gb=replay_gb, old_logp=old_logp,
                          replay_recent=int(replay_recent),
                          advantages=advantages)
    opt = DotaOptimizer(cfg, broker)
    ws = WeightStore(model, device='cpu')
    loader = ThreadPoolExecutor(1, thread_name_prefix='weights')
    if weight_lag > 0:
        # staleness on demand: the actors get version v only once `weight_lag` newer versions were published (the node
        # loop's process-mode actors run ≈12-22 versions behind; the in-process actor here ≈2-4)
        import collections
        held = collections.deque()

        def delayed(v, b):
            held.append((v, b))
            if v == 0 or len(held) > weight_lag:
                loader.submit(ws.add_bytes, *held.popleft())
        broker.subscribe_model(delayed)
    else:
        broker.subscribe_model(lambda v, b: loader.submit(ws.add_bytes, v, b))
    loader.submit(lambda: None).result()
    lg = None
    if league:
        from ..actor.league import League
        lg = League(ws, mode=league)
    va = VecActor(ws, games, broker.publish_experience, device=device, seed=seed, rollout_size=9999,
                  max_dota_time=max_dota_time, hidden_stride=seq_len, threads=threads, stagger=True, mode=mode,
                  league=lg, latest_weights_prob=latest_weights_prob if lg is not None else 1.0,
                  precision=actor_precision)
    stop, pause, paused, err = threading.Event(), threading.Event(), threading.Event(), []
    rows: List[Dict] = []
    sync = torch.cuda.synchronize if str(device).startswith('cuda') else (lambda: None)

    def actor_loop():
        try:
            while not stop.is_set():
                if pause.is_set():
                    paused.set()
                    time.sleep(0.005)
                    continue
                paused.clear()
                va.step()
        except BaseException as e:       # surfaced by the training loop
            err.append(e)
            paused.set()

    snaps: List = []                   # (t_train, cpu state_dict) at every evaluation: the snapshot pool

    def evaluate(row):
        pause.set()
        if th.is_alive():
            paused.wait(timeout=60)
        opt.flush_metrics()
        sync()
        t0 = time.time()
        row.update(evaluate_vs_default_bot(opt.policy, n_games=eval_games, device=device, seed=eval_seed,
                                           max_dota_time=max_dota_time, threads=threads, precision=eval_precision))
        t_now = float(row.get('t_train', 0.0))
        for lag in snapshot_lags or ():
            past = [sn for sn in snaps if sn[0] <= t_now - lag + 1e-6]
            if not past:
                continue
            r = evaluate_vs_snapshot(opt.policy, past[-1][1], n_games=snapshot_games, device=device,
                                     seed=eval_seed + int(lag), max_dota_time=max_dota_time, threads=threads,
                                     precision=eval_precision)
            tag = f'{int(lag) // 60}min' if lag >= 60 else f'{int(lag)}s'
            row[f'snap/win_rate_vs_{tag}'] = r['win_rate']
            row[f'snap/age_s_vs_{tag}'] = round(t_now - past[-1][0], 1)
        snaps.append((t_now, {k: v.detach().cpu().clone() for k, v in opt.policy.state_dict().items()}))
        if lg is not None:
            g = sum(lg.games.values())
            row['league/pool'] = len(ws.weights)
            row['league/score'] = sum(lg.wins.values()) / g if g else None
            row['league/games'] = g
        row['eval_s'] = round(time.time() - t0, 3)
        pause.clear()
        rows.append(row)
        if on_row is not None:
            on_row(row)

    th = threading.Thread(target=actor_loop, daemon=True)
    trained, samples, it = float(resumed.get('t_train', 0.0)), int(resumed.get('samples', 0)), opt.iteration_start
    steps0 = int(resumed.get('actor_steps', 0))
    if resumed and it - 1 != resumed.get('iteration'):
        raise RuntimeError(f'curve state at iteration {resumed.get("iteration")} but the checkpoint is {it - 1}')

    def save_state():
        if log_dir:
            with open(state_path, 'w') as fh:
                json.dump({'t_train': trained, 'samples': samples, 'actor_steps': steps0 + va.steps_taken,
                           'iteration': it - 1}, fh)
    try:
        if not resumed:
            evaluate({'t_train': 0.0, 'iteration': 0, 'samples': 0, 'actor_steps': 0, 'model': model,
                      'precision': precision, 'backend': backend, 'pack': bool(pack), 'league': league,
                      'actor_precision': actor_precision, 'replay_gb': replay_gb, 'replay_recent': int(replay_recent),
                      'advantages': advantages, 'old_logp': old_logp, 'weight_lag': int(weight_lag)})
        th.start()
        next_eval = (int(trained // eval_every) + 1) * eval_every
        while trained < budget:
            t0 = time.time()
            opt.run_iteration(it)
            it += 1
            samples += seq_per_epoch * seq_len
            trained += time.time() - t0
            if err:
                raise err[0]
            if trained >= next_eval or trained >= budget:
                m = getattr(opt, 'last_metrics', {}) or {}
                evaluate({'t_train': round(trained, 1), 'iteration': it - 1, 'samples': samples,
                          'actor_steps': steps0 + va.steps_taken, 'resumed': bool(resumed), 'loss': m.get('loss/sum'), 'entropy': m.get('entropy'),
                          'train_reward_per_sec': m.get('reward_per_sec/sum'),
                          'avg_weight_age': m.get('avg_weight_age'), 'approx_kl': m.get('approx_kl'),
                          'clipfrac': m.get('clipfrac'),
                          **{k: v for k, v in m.items() if k.startswith('offpolicy/')}})
                next_eval += eval_every
        if league_matrix_n and len(snaps) >= 2:
            # the pool's pairwise win rates: snapshots spread evenly over the run, oldest first
            from ..actor.validate import league_matrix
            pause.set()
            if th.is_alive():
                paused.wait(timeout=60)
            k = min(league_matrix_n, len(snaps))
            pick = [snaps[round(i * (len(snaps) - 1) / (k - 1))] for i in range(k)]
            lm = league_matrix([(f't{int(t)}s', sd) for t, sd in pick], opt.policy.config,
                               n_games=snapshot_games, device=device, max_dota_time=max_dota_time, threads=threads,
                               precision=eval_precision)
            row = {'league_matrix': lm, 't_train': round(trained, 1)}
            rows.append(row)
            if on_row is not None:
                on_row(row)
        if save_model:
            opt.flush_metrics()
            sync()
            torch.save({k: v.detach().cpu() for k, v in opt.policy.state_dict().items()}, save_model)
    finally:
        stop.set()
        if th.is_alive():
            th.join(timeout=60)
        opt.close()
        va.close()
        opt.flush_checkpoints()
        save_state()
        loader.shutdown(wait=True)
    return rows
