"""Eager vs graph-captured learner steps at the bench shape: parameters and losses must agree; err must be 0."""
import copy
import os
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

torch.manual_seed(0)
cfg = get_config('lstm512')
pol = Policy(cfg)
ref = copy.deepcopy(pol)
lc = LossConfig(algo='ppo')
a = Learner(pol, lc, device='cuda', backend='fused', dp=False)
b = Learner(ref, lc, device='cuda', backend='fused', dp=False)
b.enable_graph(warmup=1)
batches = [make_batch(8, 1400, cfg.layout, cfg.hidden, device='cuda', seed=s) for s in range(4)]
for i, bt in enumerate(batches):
    torch.cuda.synchronize(); t0 = time.time()
    ma = a.train_step(bt); torch.cuda.synchronize(); t1 = time.time()
    mb = b.train_step(bt); torch.cuda.synchronize(); t2 = time.time()
    print(i, 'eager %.2f ms graph %.2f ms' % ((t1 - t0) * 1e3, (t2 - t1) * 1e3), float(ma['loss']), float(mb['loss']),
          'err', int(a.model.err.item()), int(b.model.err.item()))
print('max param diff', (a.flat.flat - b.flat.flat).abs().max().item())
