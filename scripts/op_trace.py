#!/usr/bin/env python3
"""Map every GPU kernel of ONE eager fused learner step to the Python line that launched it (torch.profiler with
stacks): finds the origin of the small glue kernels seen in rocprofv3 timelines."""
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import DeviceReplay  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

dev = torch.device('cuda')
cfg = get_config('lstm512')
pol = Policy(cfg)
learner = Learner(pol, LossConfig(algo='ppo'), device=dev, backend='fused')
rep = DeviceReplay(32, 1400, cfg.layout, cfg.hidden, dev, seed=0)
for _ in range(2):
    learner.train_step(rep.sample(8))
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    learner.train_step(rep.sample(8))
    torch.cuda.synchronize()
n = 0
for e in prof.events():
    if e.device_type != torch.autograd.DeviceType.CPU or not e.kernels:
        continue
    if any(c.kernels for c in e.cpu_children):
        continue
    frames = [f for f in (e.stack or []) if 'dotaclient_amd' in f or 'bench' in f]
    where = frames[0].split('/')[-1] if frames else '?'
    for k in e.kernels:
        n += 1
        print(f'{n:4d} {k.duration:8.1f} {e.name[:28]:28s} {where[:60]:60s} {k.name[:50]}')
