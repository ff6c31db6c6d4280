"""Per-tensor gradient comparison fused vs torch-fp32 for a preset (debug helper)."""
import copy
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else '5v5'
torch.manual_seed(0)
cfg = get_config(preset)
pol = Policy(cfg)
ref = copy.deepcopy(pol)
lc = LossConfig(algo='ppo', vf_coef=0.5, entropy_coef=0.01)
fused = Learner(pol, lc, device='cuda', backend='fused', dp=False)
tl = Learner(ref, lc, device='cuda', backend='torch', dp=False)
tl.backend = 'torch-fp32'
batch = make_batch(3, 24, cfg.layout, cfg.hidden if cfg.rnn == 'lstm' else None, device='cuda', seed=3)
for L in (fused, tl):
    L.dp.zero_grad()
lf, _ = fused.loss(batch)
lf.backward()
lr, _ = tl.loss(batch)
lr.backward()
torch.cuda.synchronize()
print('loss', float(lf), float(lr))
for name, a, b in zip(fused.flat.names, [p.grad for p in fused.flat.params], [p.grad for p in tl.flat.params]):
    if a is None or b is None:
        print(f'{name:40s} missing grad fused={a is not None} ref={b is not None}')
        continue
    rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
    print(f'{name:40s} rel={rel:.4f} |ref|={b.norm().item():.3e} |fused|={a.norm().item():.3e}')
