"""Run presets: the five BASELINE.json configurations as named bundles of flags for every entrypoint.

``--preset NAME`` on ``cli/optimizer.py``, ``cli/agent.py``, ``cli/launch.py`` and ``bench.py`` sets that role's
defaults (explicit flags still win — the preset only changes what an omitted flag means). The reference configures
its one deployment through ks-app params (params.libsonnet:7-24: batch 8, seq_len 1400, 16 sequences/iteration,
1 epoch, rollout size 9999, max dota time 600); these presets extend that to the configurations the MI355X build
is measured on.

=====================  =======================================================================================
preset                 BASELINE.json config
=====================  =======================================================================================
``cpu-plumbing``       1 — 1v1-mid single actor + CPU optimizer, LSTM-128, synthetic obs (no GPU)
``lstm512-1gpu``       2 — 1v1-mid LSTM-512, batched actor inference + PPO on 1 MI355X
``lstm512-8gpu``       3 — 1v1-mid LSTM-512, 8×MI355X data-parallel optimizer (RCCL over xGMI)
``5v5-8gpu``           4 — 5v5 entity-attention policy (per-unit embed + max-pool), 8×MI355X DP
``league-replay``      5 — self-play league (PFSP) + 200 GB on-HBM replay per GPU, fp8 actor policy step
                       (``--actor-precision fp8``: actor/batched.py Fp8ActorPolicy, ops/csrc/actor_fp8.hip)
=====================  =======================================================================================
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass, field
from typing import Dict, List, Optional

_DEPLOY = dict(batch_size=8, seq_len=1400, seq_per_epoch=16, epochs=1)      # params.libsonnet:7-24


@dataclass(frozen=True)
class RunPreset:
    name: str
    config: str                                   # the BASELINE.json configuration it reproduces
    world_size: int                               # learner ranks (one per GPU)
    optimizer: Dict[str, object] = field(default_factory=dict)   # cli/optimizer.py argparse dests
    agent: Dict[str, object] = field(default_factory=dict)       # cli/agent.py argparse dests
    bench: Dict[str, object] = field(default_factory=dict)       # bench.py argparse dests
    launch: Dict[str, object] = field(default_factory=dict)      # cli/launch.py argparse dests


PRESETS: Dict[str, RunPreset] = {p.name: p for p in [
    RunPreset('cpu-plumbing', '1v1-mid single actor + CPU optimizer, LSTM-128 policy on synthetic obs', 1,
              optimizer=dict(model_preset='lstm128', device='cpu', backend='torch', batch_size=4, seq_len=256,
                             seq_per_epoch=16, epochs=4),
              agent=dict(model_preset='lstm128', device='cpu', games=1, runtime='service'),
              bench=dict(model='lstm128', batch_size=4, seq_len=256),
              launch=dict(model_preset='lstm128', actors=1, games_per_actor=1, actor_device='cpu', optimizers=1)),
    RunPreset('lstm512-1gpu', '1v1-mid LSTM-512 policy, batched actor inference + PPO on 1 MI355X', 1,
              optimizer=dict(model_preset='lstm512', precision='fp32-exact', **_DEPLOY),
              agent=dict(model_preset='lstm512', device='cuda', games=1024, runtime='vec', rollout_size=9999,
                         max_dota_time=600),
              bench=dict(model='lstm512', batch_size=8, seq_len=1400, precision='fp32-exact'),
              launch=dict(model_preset='lstm512', actors=1, games_per_actor=1024, actor_device='cuda',
                          optimizers=1)),
    RunPreset('lstm512-8gpu', '1v1-mid LSTM-512, 8xMI355X data-parallel optimizer with RCCL all-reduce over xGMI', 8,
              optimizer=dict(model_preset='lstm512', precision='fp32-exact', **_DEPLOY),
              agent=dict(model_preset='lstm512', device='cuda', games=1024, runtime='vec', rollout_size=9999,
                         max_dota_time=600),
              bench=dict(model='lstm512', batch_size=8, seq_len=1400, precision='fp32-exact'),
              launch=dict(model_preset='lstm512', actors=8, games_per_actor=1024, actor_device='cuda',
                          optimizers=8)),
    RunPreset('5v5-8gpu', '5v5 entity-attention policy (per-unit embed + max-pool), 8xMI355X DP', 8,
              optimizer=dict(model_preset='5v5', precision='fp32', **_DEPLOY),
              agent=dict(model_preset='5v5', device='cuda', games=256, runtime='vec', rollout_size=9999,
                         max_dota_time=600),
              bench=dict(model='5v5', batch_size=8, seq_len=1400, precision='fp32'),
              launch=dict(model_preset='5v5', actors=8, games_per_actor=256, actor_device='cuda', optimizers=8)),
    RunPreset('league-replay', 'Self-play league (PFSP opponents) + 200 GB on-HBM replay buffer', 1,
              # (the learner samples the replay's 4 096 newest sequences: uniform sampling over the whole buffer
              # trained mostly on old games and learned the default-bot game several times slower,
              # profiles/r6_curve_league{,_recent}.jsonl)
              optimizer=dict(model_preset='lstm512', precision='fp32-exact', replay_gb=200.0, replay_recent=4096,
                             **_DEPLOY),
              agent=dict(model_preset='lstm512', device='cuda', games=1024, runtime='vec', rollout_size=9999,
                         max_dota_time=600, league='pfsp', use_latest_weights_prob=0.8, actor_precision='fp8'),
              bench=dict(model='lstm512', batch_size=8, seq_len=1400, precision='fp32-exact', replay=16384),
              launch=dict(model_preset='lstm512', actors=1, games_per_actor=1024, actor_device='cuda',
                          optimizers=1)),
]}


def get_preset(name: str) -> RunPreset:
    if name not in PRESETS:
        raise ValueError(f'unknown preset {name!r}; one of {sorted(PRESETS)}')
    return PRESETS[name]


def add_preset_arg(ap: argparse.ArgumentParser):
    ap.add_argument('--preset', type=str, default=None, choices=sorted(PRESETS),
                    help='run preset (BASELINE configs 1-5) setting this role\'s defaults; explicit flags win')


def parse_with_preset(ap: argparse.ArgumentParser, role: str, argv: Optional[List[str]] = None):
    """Parse ``argv`` with the role's preset values as defaults (``--preset`` must be registered on ``ap``)."""
    pre, _ = ap.parse_known_args(argv)
    if getattr(pre, 'preset', None):
        values = dict(getattr(get_preset(pre.preset), role))
        known = {a.dest for a in ap._actions}
        unknown = set(values) - known
        if unknown:
            raise ValueError(f'preset {pre.preset!r} sets unknown {role} options {sorted(unknown)}')
        ap.set_defaults(**values)
    return ap.parse_args(argv)
