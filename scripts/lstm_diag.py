"""Team-LSTM forward (fp32 weights, precise activations: the fp32-exact learner's recurrence) vs a float64 and a
float32 torch loop, B=8, S=1400, H=512: error of h over the horizon. python scripts/lstm_diag.py"""
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.ops.lstm import team_fwd  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def loop(xp, whh, h0, c0):
    S = xp.shape[0]
    h, c = h0, c0
    hs = []
    for t in range(S):
        g = xp[t] + h @ whh.t()
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        hs.append(h)
    return torch.stack(hs)


C = ops.require()
S, B, H = 1400, 8, 512
g = torch.Generator(device='cuda').manual_seed(0)
k = H ** -0.5
whh = (torch.rand(4 * H, H, device='cuda', generator=g) * 2 - 1) * k
xp = torch.randn(S, B, 4 * H, device='cuda', generator=g) * 0.5
h0 = torch.zeros(B, H, device='cuda')
c0 = torch.zeros(B, H, device='cuda')
err = torch.zeros(1, dtype=torch.int32, device='cuda')
h64 = loop(xp.double(), whh.double(), h0.double(), c0.double())
h32 = loop(xp, whh, h0, c0)
xp4 = xp.view(S, B, 4, H).transpose(2, 3).contiguous()
for prec in (True, False):
    o = team_fwd(C, xp4, whh, h0, c0, err, False, time_major=True, precise=prec)
    hs = o[0].float()
    torch.cuda.synchronize()
    print(f'precise={prec} err={int(err.item())} kernel vs fp64: all {rel(hs, h64):.3e}  '
          + '  '.join(f't{t}: {rel(hs[t], h64[t]):.2e}' for t in (0, 10, 100, 700, 1399)), flush=True)
print(f'torch fp32 loop vs fp64: all {rel(h32, h64):.3e}  '
      + '  '.join(f't{t}: {rel(h32[t], h64[t]):.2e}' for t in (0, 10, 100, 700, 1399)), flush=True)
