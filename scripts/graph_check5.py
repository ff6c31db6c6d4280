"""Debug: graph loop WITHOUT per-step host sync (bench-like); losses printed at the end."""
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import DeviceReplay  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else 'nosync'
torch.manual_seed(int(__import__('os').environ.get('SEED', '0')))
cfg = get_config('lstm512')
import os
DEV = torch.device(os.environ.get('DEV', 'cuda'))
if DEV.index is not None:
    torch.cuda.set_device(DEV)
L = Learner(Policy(cfg), LossConfig(algo='ppo'), device=DEV, backend='fused', dp=os.environ.get('DP') == '1')
L.enable_graph(warmup=1)
rp = DeviceReplay(32, 1400, cfg.layout, cfg.hidden, DEV, seed=0)
ms = []
torch.cuda.synchronize()
t0 = time.time()
for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 8):
    bt = rp.sample(8)
    t1 = time.time()
    ms.append(L.train_step(bt))
    if mode in ('sync', 'gc'):
        torch.cuda.synchronize()
        if mode == 'gc' and i == 3:
            import gc
            print('gc collected', gc.collect(), flush=True)
        print(i, 'step ms %.2f' % ((time.time() - t1) * 1e3), float(ms[-1]['loss']), 'gnorm', float(ms[-1]['grad_norm']), 'err', int(L.model.err.item()), flush=True)
torch.cuda.synchronize()
print(mode, 'total ms %.1f' % ((time.time() - t0) * 1e3))
for i, m in enumerate(ms):
    print(i, float(m['loss']), float(m['grad_norm']))
print('param finite', bool(torch.isfinite(L.flat.flat).all()), 'err', int(L.model.err.item()))
