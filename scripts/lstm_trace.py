#!/usr/bin/env python3
"""In-kernel timestamps of the persistent LSTM forward (s_memrealtime, 10 ns): where a recurrence step's time goes.
Events per (workgroup, wave, step): 0 poll start, 1 probe ok, 2 fetch ok, 3 pre-barrier (pollers); 4 post-barrier,
5 h_t published (publisher). Prints median phase durations and the cross-workgroup hand-off latency."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402


def main(B=8, H=512, S=200):
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
        C.lstm_fwd(xp, whh, h0, h0, err, False, tr)
    torch.cuda.synchronize()
    t = tr.view(nwg, 8, 64, 8).cpu().numpy().astype(np.float64) * 10.0   # ns
    steps = slice(8, 60)
    pol = t[:, 0:4, steps]        # pollers
    pub = t[:, 4, steps]          # publisher
    out = {'B': B, 'H': H}
    step_ns = np.diff(pub[:, :, 4], axis=1)
    out['step_ns_median'] = float(np.median(step_ns))
    out['probe_wait_ns'] = float(np.median(pol[..., 1] - pol[..., 0]))
    out['fetch_ns'] = float(np.median(pol[..., 2] - pol[..., 1]))
    out['mfma_lds_ns'] = float(np.median(pol[..., 3] - pol[..., 2]))
    out['barrier_to_publisher_ns'] = float(np.median(pub[..., 4] - pol[..., 3].max(axis=1)))
    out['publisher_ns'] = float(np.median(pub[..., 5] - pub[..., 4]))
    # hand-off: last publisher store of step t (over all WGs) → earliest probe success of step t+1
    last_pub = pub[..., 5].max(axis=0)               # per step
    first_probe = pol[..., 1].min(axis=(0, 1))
    out['publish_to_first_probe_ns'] = float(np.median(first_probe[1:] - last_pub[:-1]))
    last_probe = pol[..., 1].max(axis=(0, 1))
    out['publish_to_last_probe_ns'] = float(np.median(last_probe[1:] - last_pub[:-1]))
    out['err'] = int(err.item())
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    for B in (8, 32):
        main(B=B)
    main(B=8, H=128)
