"""Validation against the scripted default bot on the native vectorised engine — the reference's only quality signal.

The reference runs a separate validation agent (``--validation``, /root/reference/agent.py:905-927): its hero plays
the Dota default bot (``HERO_CONTROL_MODE_DEFAULT``) with the latest weights, sends no experience, and writes
``game/rewards_sum`` / ``game/rewards_<key>`` (and the canvas) to tensorboard per game (agent.py:415-434). Here the
same evaluation runs many games at once: :class:`~dotaclient_amd.actor.vec.VecActor` in ``vs_default_bot`` mode (the
controlled side alternates between Radiant and Dire with the game serial; the bot is ``native/vecenv.h``
``default_bot``, bit-identical to ``env/synthetic.py:256-276``), every finished game's trajectory is decoded from its
rollout message and reduced to the reference's metrics plus the win rate (end-state reward +1 win / −1 loss / −0.25
time limit, agent.py:325-337).
"""
from __future__ import annotations

import time
from typing import Dict, List

import numpy as np

from ..constants import REWARD_KEYS


def evaluate_vs_default_bot(policy, n_games: int = 128, device='cuda', seed: int = 12345,
                            max_dota_time: float = 600.0, threads: int = 8, timeout: float = 600.0,
                            precision: str = 'fp32') -> Dict[str, float]:
    """Play ``n_games`` games of ``policy`` (a :class:`~dotaclient_amd.models.policy.Policy`) against the default bot
    and return the reference's validation metrics averaged over the games: ``game/rewards_sum``,
    ``game/rewards_<key>`` for every reward key, ``game/win_rate`` (wins / games), ``game/loss_rate``,
    ``game/steps`` (mean game length) and ``games``. A fixed ``seed`` gives the same games for every policy.
    ``precision``: the policy step the games are played with — by default the IEEE-fp32 actor
    (:class:`~dotaclient_amd.actor.batched.F32ActorPolicy`, the weights as the learner trained them; the reference's
    validation agent runs the fp32 policy); 5v5 policies fall back to bf16 operands."""
    from ..transport.codec import decode
    from .vec import VecActor
    from .weights import WeightStore

    ws = WeightStore(policy.config, device='cpu')
    ws.add(0, {k: v.detach().cpu() for k, v in policy.state_dict().items()})
    msgs: List[bytes] = []
    mode = 'vs_default_bot_5v5' if policy.config.layout.counts[0] > 1 else 'vs_default_bot'   # 5 heroes a side
    va = VecActor(ws, n_games, msgs.append, device=device, mode=mode, seed=seed,
                  rollout_size=10 ** 9, max_dota_time=max_dota_time, threads=threads, groups=1, stagger=False,
                  tag=f'val{seed}', precision=precision)
    t0 = time.time()
    try:
        while va.games_finished < n_games:
            va.step()
            if time.time() - t0 > timeout:
                raise TimeoutError(f'validation: {va.games_finished}/{n_games} games after {timeout:.0f} s')
    finally:
        va.close()
    per_game: Dict[str, List[float]] = {}
    for body in msgs:
        r = decode(body)
        rew = np.asarray(r.rewards, np.float64)
        per_game.setdefault(r.game_id, [])
        sums = rew.sum(axis=0)
        row = {k: float(v) for k, v in zip(REWARD_KEYS, sums)}
        row.update({'sum': float(sums.sum()), 'steps': float(rew.shape[0]), 'won': float(rew[-1, 1] > 0.5),
                    'lost': float(rew[-1, 1] < -0.5)})
        per_game[r.game_id].append(row)
    # one controlled player per game (5v5: the team's rewards are per player; the end state is shared)
    games = [rows[0] for rows in list(per_game.values())[:n_games]]
    out: Dict[str, float] = {'games': float(len(games))}
    if not games:
        return out
    mean = lambda k: float(np.mean([g[k] for g in games]))             # noqa: E731
    out['game/rewards_sum'] = mean('sum')
    out['game/win_rate'] = mean('won')
    out['game/loss_rate'] = mean('lost')
    out['game/steps'] = mean('steps')
    for k in REWARD_KEYS:
        out[f'game/rewards_{k}'] = mean(k)
    return out



def evaluate_vs_snapshot(policy, snapshot_state, n_games: int = 64, device='cuda', seed: int = 777,
                         max_dota_time: float = 600.0, threads: int = 8, timeout: float = 900.0,
                         precision: str = 'fp32') -> Dict[str, float]:
    """Head-to-head games of ``policy`` (the current weights) against a frozen past snapshot of the same network
    (``snapshot_state``: a state_dict) — the discriminating signal once the default-bot win rate saturates, and one
    entry of the league's win-rate matrix. Every game is a league game of the self-play engine (VecActor with
    ``latest_weights_prob`` 0: one team — Radiant or Dire at random — plays the snapshot, the other the current
    weights; reference mini-league, agent.py:760-765); a fixed ``seed`` replays the same openings. Returns
    ``win_rate`` (wins + ½ time-limit draws, per game), ``wins`` / ``losses`` / ``draws`` and ``games``."""
    from .league import League
    from .vec import VecActor
    from .weights import WeightStore

    ws = WeightStore(policy.config, device='cpu')
    ws.add(0, {k: v.detach().cpu() for k, v in snapshot_state.items()})
    ws.add(1, {k: v.detach().cpu() for k, v in policy.state_dict().items()})
    lg = League(ws, mode='oldest')
    mode = '5v5' if policy.config.layout.counts[0] > 1 else '1v1'
    va = VecActor(ws, n_games, None, device=device, mode=mode, seed=seed, rollout_size=10 ** 9,
                  max_dota_time=max_dota_time, threads=threads, groups=1, stagger=False, league=lg,
                  latest_weights_prob=0.0, opponent_refresh=10 ** 9, tag=f'snap{seed}', precision=precision)
    t0 = time.time()
    try:
        while lg.games.get(0, 0.0) < n_games:
            va.step()
            if time.time() - t0 > timeout:
                raise TimeoutError(f'snapshot evaluation: {lg.games.get(0, 0.0):.0f}/{n_games} games after '
                                   f'{timeout:.0f} s')
    finally:
        va.close()
    games = lg.games.get(0, 0.0)
    score = lg.wins.get(0, 0.0)
    res = getattr(lg, 'results', {}).get(0, [])
    out = {'games': float(games), 'win_rate': score / max(games, 1.0)}
    if res:
        out.update(wins=float(sum(1 for r in res if r == 1.0)), losses=float(sum(1 for r in res if r == 0.0)),
                   draws=float(sum(1 for r in res if r == 0.5)))
    return out


def league_matrix(snapshots, config, n_games: int = 32, device='cuda', seed: int = 991, max_dota_time: float = 600.0,
                  threads: int = 8, precision: str = 'fp32') -> Dict[str, object]:
    """Pairwise win rates of league snapshots ``[(label, state_dict), …]`` (oldest first): entry [i][j] is the
    score of snapshot i against snapshot j over ``n_games`` games (wins + ½ draws; [j][i] = 1 − [i][j]). A healthy
    league is (mostly) increasing along each row's diagonal direction: later snapshots beat earlier ones."""
    from ..models.policy import Policy
    labels = [lab for lab, _ in snapshots]
    n = len(snapshots)
    m = [[0.5] * n for _ in range(n)]
    for i in range(n):
        pol = Policy(config)
        pol.load_state_dict(snapshots[i][1])
        for j in range(i):
            r = evaluate_vs_snapshot(pol, snapshots[j][1], n_games=n_games, device=device, seed=seed + 31 * i + j,
                                     max_dota_time=max_dota_time, threads=threads, precision=precision)
            m[i][j] = r['win_rate']
            m[j][i] = 1.0 - r['win_rate']
    return {'labels': labels, 'win_rate': m, 'games_per_pair': n_games}
