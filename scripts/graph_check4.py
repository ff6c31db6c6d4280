"""Debug: bench-like loop with graph capture; print per-step loss / grad norm / param finiteness."""
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import DeviceReplay  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

torch.manual_seed(0)
cfg = get_config('lstm512')
L = Learner(Policy(cfg), LossConfig(algo='ppo'), device='cuda', backend='fused', dp=False)
L.enable_graph(warmup=1)
rp = DeviceReplay(32, 1400, cfg.layout, cfg.hidden, 'cuda', seed=0)
for i in range(6):
    bt = rp.sample(8)
    torch.cuda.synchronize()
    t0 = time.time()
    m = L.train_step(bt)
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(i, 'ms %.2f' % (dt * 1e3), 'loss', float(m['loss']), 'gnorm', float(m['grad_norm']),
          'grad finite', bool(torch.isfinite(L.flat.grad).all()), 'param finite', bool(torch.isfinite(L.flat.flat).all()),
          'counts', float(L.dp.counts.sum()), 'err', int(L.model.err.item()), flush=True)
