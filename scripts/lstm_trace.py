#!/usr/bin/env python3
"""In-kernel timestamps of the persistent LSTM kernels (s_memrealtime, 10 ns): where a recurrence step's time goes.

Forward events per (workgroup, wave, step): 0 poll start, 1 poll ok, 2 fragments decoded, 3 pre-barrier (pollers);
4 post-barrier, 6 h_t granules stored, 5 outputs stored (publisher).
Backward: 0 poll start, 1 poll ok, 2 pre-barrier (pollers); 3 post-barrier, 4 gate grads, 5 partials stored,
6 ∂gates stored (publishers). Prints median phase durations and the cross-workgroup hand-off latency."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402

med = (lambda a: float(np.median(a)))


def fwd(B=8, H=512, S=200):
    C = ops.require()
    torch.manual_seed(0)
    xp = torch.randn(B, S, 4 * H, device='cuda') * 0.5
    whh = (torch.randn(4 * H, H, device='cuda') * 0.05).to(torch.bfloat16)
    h0 = torch.zeros(B, H, device='cuda')
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    nwg = H // 8
    tr = torch.zeros(nwg * 8 * 64 * 8, dtype=torch.int64, device='cuda')
    for _ in range(3):
        tr.zero_()
        out = C.lstm_fwd(xp, whh, h0, h0, err, False, tr)
    torch.cuda.synchronize()
    t = tr.view(nwg, 8, 64, 8).cpu().numpy().astype(np.float64) * 10.0   # ns
    steps = slice(8, 60)
    pol = t[:, 0:4, steps]
    pub = t[:, 4, steps]
    o = {'kernel': 'fwd', 'B': B, 'H': H}
    o['step_ns'] = med(np.diff(pub[:, :, 4], axis=1))
    o['poll_wait_ns'] = med(pol[..., 1] - pol[..., 0])
    o['decode_ns'] = med(pol[..., 2] - pol[..., 1])
    o['mfma_lds_ns'] = med(pol[..., 3] - pol[..., 2])
    o['barrier_ns'] = med(pub[..., 4] - pol[..., 3].max(axis=1))
    o['pub_compute_ns'] = med(pub[..., 6] - pub[..., 4])
    o['pub_outputs_ns'] = med(pub[..., 5] - pub[..., 6])
    last_pub = pub[..., 6].max(axis=0)
    o['granule_to_first_poll_ok_ns'] = med(pol[..., 1].min(axis=(0, 1))[1:] - last_pub[:-1])
    o['granule_to_last_poll_ok_ns'] = med(pol[..., 1].max(axis=(0, 1))[1:] - last_pub[:-1])
    o['err'] = int(err.item())
    print(json.dumps(o), flush=True)
    return out


def bwd(B=8, H=512, S=200):
    C = ops.require()
    torch.manual_seed(0)
    xp = torch.randn(B, S, 4 * H, device='cuda') * 0.5
    whh = (torch.randn(4 * H, H, device='cuda') * 0.05).to(torch.bfloat16)
    h0 = torch.zeros(B, H, device='cuda')
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    out = C.lstm_fwd(xp, whh, h0, h0, err, False)
    dh = torch.randn(B, S, H, device='cuda')
    nwg = H // 8
    tr = torch.zeros(nwg * 8 * 64 * 8, dtype=torch.int64, device='cuda')
    for _ in range(3):
        tr.zero_()
        C.lstm_bwd(dh, out[3], out[2], h0, None, None, whh, err, tr)
    torch.cuda.synchronize()
    t = tr.view(nwg, 8, 64, 8).cpu().numpy().astype(np.float64) * 10.0
    steps = slice(8, 60)
    pol = t[:, 0:4, steps]
    pub = t[:, 4:8, steps]
    o = {'kernel': 'bwd', 'B': B, 'H': H}
    o['step_ns'] = med(np.diff(pub[:, 0, :, 3], axis=1))
    o['poll_wait_ns'] = med(pol[..., 1] - pol[..., 0])
    o['prefetch_lds_ns'] = med(pol[..., 2] - pol[..., 1])
    o['barrier_ns'] = med(pub[..., 3].min(axis=1) - pol[..., 2].max(axis=1))
    o['gate_grads_ns'] = med(pub[..., 4] - pub[..., 3])
    o['mfma_stores_ns'] = med(pub[..., 5] - pub[..., 4])
    o['dgates_ns'] = med(pub[..., 6] - pub[..., 5])
    last_pub = pub[..., 5].max(axis=(0, 1))
    o['partials_to_first_poll_ok_ns'] = med(pol[..., 1].min(axis=(0, 1))[1:] - last_pub[:-1])
    o['partials_to_last_poll_ok_ns'] = med(pol[..., 1].max(axis=(0, 1))[1:] - last_pub[:-1])
    o['err'] = int(err.item())
    print(json.dumps(o), flush=True)


if __name__ == '__main__':
    for B, H in ((8, 512), (8, 128)):
        fwd(B=B, H=H)
        bwd(B=B, H=H)
