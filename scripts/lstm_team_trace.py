#!/usr/bin/env python3
"""In-kernel timestamps (s_memrealtime, 10 ns) of the XCD-team LSTM forward: per-step phase breakdown.
Events per (member workgroup, wave, step): 0 step start, 1 h_{t-1} gathered, 2 after barrier, 3 gates/transposed,
4 h_t published, 5 outputs stored. ``f32`` in argv: the fp32 (bf16x3) kernel variant (fp32 W_hh)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.ops.lstm import team_ctl  # noqa: E402

med = (lambda a: float(np.median(a)))
F32 = 'f32' in sys.argv
WDT = torch.float32 if F32 else torch.bfloat16


def fwd(B=8, H=512, S=200):
    C = ops.require()
    torch.manual_seed(0)
    xp = torch.randn(B, S, H, 4, device='cuda') * 0.5
    whh = (torch.randn(4 * H, H, device='cuda') * 0.05).to(WDT)
    h0 = torch.zeros(B, H, device='cuda')
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    tr = torch.zeros(32 * 4 * 64 * 8, dtype=torch.int64, device='cuda')
    for _ in range(3):
        tr.zero_()
        C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), False, tr)
    torch.cuda.synchronize()
    t = tr.view(32, 4, 64, 8).cpu().numpy().astype(np.float64) * 10.0
    nt = H // 128
    w = t[:, :nt, 8:60]                     # MFMA waves
    o = {'kernel': 'team_fwd', 'f32': F32, 'B': B, 'H': H}
    o['step_ns'] = med(np.diff(w[..., 0], axis=2))
    o['gather_ns'] = med(w[..., 1] - w[..., 0])
    o['barrier_ns'] = med(w[..., 2] - w[..., 1])
    o['mfma_cell_ns'] = med(w[..., 3] - w[..., 2])
    o['publish_ns'] = med(w[..., 4] - w[..., 3])
    o['outputs_ns'] = med(w[..., 5] - w[..., 4])
    last_pub = w[..., 4].max(axis=(0, 1))
    o['publish_to_first_gather_ns'] = med(w[..., 1].min(axis=(0, 1))[1:] - last_pub[:-1])
    o['publish_to_last_gather_ns'] = med(w[..., 1].max(axis=(0, 1))[1:] - last_pub[:-1])
    first_pub = w[..., 4].min(axis=(0, 1))
    o['publish_skew_ns'] = med(last_pub - first_pub)
    o['err'] = int(err.item())
    print(json.dumps(o), flush=True)


if __name__ == '__main__' and 'bwd' not in sys.argv:
    fwd(8, 512)
    fwd(8, 128)
    if not F32:
        fwd(32, 512)


def bwd(B=8, H=512, S=200):
    C = ops.require()
    torch.manual_seed(0)
    xp = torch.randn(B, S, H, 4, device='cuda') * 0.5
    whh = (torch.randn(4 * H, H, device='cuda') * 0.05).to(WDT)
    h0 = torch.zeros(B, H, device='cuda')
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    out = C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), False)
    dh = torch.randn(B, S, H, device='cuda')
    tr = torch.zeros(32 * 4 * 64 * 8, dtype=torch.int64, device='cuda')
    for _ in range(3):
        tr.zero_()
        C.lstm_team_bwd(dh, out[3], out[2], h0, None, None, whh, err, team_ctl(), tr)
    torch.cuda.synchronize()
    t = tr.view(32, 4, 64, 8).cpu().numpy().astype(np.float64) * 10.0
    w = t[:, :, 8:60]
    o = {'kernel': 'team_bwd', 'f32': F32, 'B': B, 'H': H}
    o['step_ns'] = med(np.diff(w[..., 0], axis=2))
    o['gather_ns'] = med(w[..., 1] - w[..., 0])
    o['barrier1_ns'] = med(w[..., 2] - w[..., 1])
    # kernel events (lstm_team_bwd_body): 0 step start, 1 dG_{t+1} gathered, 2 after barrier, 3 partial recurrent
    # product done, 4 after the reduction barrier, 6 gate gradients computed + dG_t published + ∂gates stored
    # (event 5 is not stamped: reading it gave the round-2 trace's garbage ±1e15 values)
    o['recurrent_dot_ns'] = med(w[..., 3] - w[..., 2])
    o['barrier2_ns'] = med(w[..., 4] - w[..., 3])
    o['gates_publish_ns'] = med(w[..., 6] - w[..., 4])
    last_pub = w[..., 6].max(axis=(0, 1))
    o['publish_skew_ns'] = med(last_pub - w[..., 6].min(axis=(0, 1)))
    o['publish_to_first_gather_ns'] = med(w[..., 1].min(axis=(0, 1))[1:] - last_pub[:-1])
    o['publish_to_last_gather_ns'] = med(w[..., 1].max(axis=(0, 1))[1:] - last_pub[:-1])
    o['err'] = int(err.item())
    print(json.dumps(o), flush=True)


if __name__ == '__main__' and 'bwd' in sys.argv:
    bwd(8, 512)
