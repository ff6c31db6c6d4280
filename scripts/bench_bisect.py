"""Bisect the bench warmup→timed transition for graph-mode gradient corruption."""
import os
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import DeviceReplay  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

V = os.environ.get('V', 'full')
device = torch.device('cuda:0')
torch.cuda.set_device(device)
torch.manual_seed(7)
cfg = get_config('lstm512')
policy = Policy(cfg)
learner = Learner(policy, LossConfig(algo='ppo'), device=device, backend='fused')
learner.enable_graph(warmup=1)
replay = DeviceReplay(32, 1400, cfg.layout, cfg.hidden, device, seed=0)


def step():
    batch = replay.sample(8)
    out = learner.train_step(batch)
    torch.cuda.synchronize()
    print(V, 'step', learner.n_steps, float(out['loss']), float(out['grad_norm']), flush=True)
    return out


for _ in range(3):
    m = step()
if V in ('full', 'nofloat'):
    torch.cuda.synchronize()
if V in ('full', 'nosync'):
    loss_val = float(m['loss'])
if V == 'keep':
    keep = m
for _ in range(3):
    m = step()
