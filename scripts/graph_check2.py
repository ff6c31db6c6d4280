"""Debug: eager vs graph grads after the first replay (non-pipelined path)."""
import copy
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1400
torch.manual_seed(0)
cfg = get_config('lstm512')
pol = Policy(cfg)
ref = copy.deepcopy(pol)
lc = LossConfig(algo='ppo')
a = Learner(pol, lc, device='cuda', backend='fused', dp=False)
b = Learner(ref, lc, device='cuda', backend='fused', dp=False)
b.enable_graph(warmup=1)
batches = [make_batch(8, S, cfg.layout, cfg.hidden, device='cuda', seed=s) for s in range(3)]
for i, bt in enumerate(batches):
    ma = a._fwd_bwd(bt)
    if i == 0:
        mb = b._fwd_bwd(bt)
    else:
        mb = b._graphed_fwd_bwd(bt)
    torch.cuda.synchronize()
    ga, gb = a.flat.grad, b.flat.grad
    print(i, 'loss', float(ma['loss']), float(mb['loss']), 'grad finite', bool(torch.isfinite(gb).all()),
          'max grad diff', (ga - gb).abs().max().item(), 'rel', ((ga - gb).norm() / ga.norm()).item())
    for nm, o, n in zip(b.flat.names, b.flat.offsets, b.flat.numel):
        d = (ga[o:o + n] - gb[o:o + n]).norm() / (ga[o:o + n].norm() + 1e-12)
        if d > 1e-3 or not torch.isfinite(gb[o:o + n]).all():
            print('   ', nm, float(d), bool(torch.isfinite(gb[o:o + n]).all()))
    # identical optimizer steps on both
    a.dp.sync(); a.opt.step(a.dp.counts)
    b.dp.sync(); b.opt.step(b.dp.counts)
torch.cuda.synchronize()
print('err', int(a.model.err.item()), int(b.model.err.item()))
