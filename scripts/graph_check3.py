"""Debug: graph replays of the same input must give identical grads, even after unrelated eager allocations."""
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1400
torch.manual_seed(0)
cfg = get_config('lstm512')
b = Learner(Policy(cfg), LossConfig(algo='ppo'), device='cuda', backend='fused', dp=False)
b.enable_graph(warmup=1)
bt = make_batch(8, S, cfg.layout, cfg.hidden, device='cuda', seed=1)
b._fwd_bwd(bt)
g0 = b.flat.grad.clone()
m = b._graphed_fwd_bwd(bt)
torch.cuda.synchronize()
g1 = b.flat.grad.clone()
print('capture+replay vs eager', (g1 - g0).abs().max().item(), float(m['loss']))
m = b._graphed_fwd_bwd(bt)
torch.cuda.synchronize()
print('replay 2', (b.flat.grad - g1).abs().max().item(), float(m['loss']))
junk = [torch.full((1 << 26,), float('nan'), device='cuda') for _ in range(8)]
del junk
torch.cuda.synchronize()
m = b._graphed_fwd_bwd(bt)
torch.cuda.synchronize()
print('replay after NaN-filled allocations', (b.flat.grad - g1).abs().max().item(), float(m['loss']))
junk = [torch.full((1 << 20,) , float('nan'), device='cuda') for _ in range(200)]
m = b._graphed_fwd_bwd(bt)
torch.cuda.synchronize()
print('replay with live small NaN allocations', (b.flat.grad - g1).abs().max().item(), float(m['loss']))
print('err', int(b.model.err.item()))
