#!/usr/bin/env python3
"""A/B of the team LSTM's merged output stores (default) against the three-store form (DCA_TEAM_KNOBS bit 14) at the
learner shape (fp32 W_hh, B=8, S=1400, H=512, time-major, folded bias): interleaved rounds in one process, per-step
µs of forward and backward, and a bitwise comparison of every output (the two forms compute the same values; only
which lanes store them differs)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.ops.lstm import team_ctl  # noqa: E402


def run(C, xp, whh, h0, c0, err, b4, dh, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(reps):
        ev[0].record()
        f = C.lstm_team_fwd(xp, whh, h0, c0, err, team_ctl(), False, None, True, None, None, None, b4, False)
        ev[1].record()
        b = C.lstm_team_bwd(dh, f[3], f[2], c0, None, None, whh, err, team_ctl(), None, True, None, False, True, False)
        ev[2].record()
        torch.cuda.synchronize()
        tf += ev[0].elapsed_time(ev[1])
        tb += ev[1].elapsed_time(ev[2])
    return f, b, tf / reps, tb / reps


def main():
    C = ops.require()
    B, S, H = 8, 1400, 512
    torch.manual_seed(0)
    dev = 'cuda'
    xp = torch.randn(S, B, H, 4, device=dev) * 0.5
    whh = torch.randn(4 * H, H, device=dev) * 0.05
    h0 = torch.randn(B, H, device=dev) * 0.1
    c0 = torch.randn(B, H, device=dev) * 0.1
    b4 = torch.randn(4 * H, device=dev) * 0.1
    dh = torch.randn(S, B, H, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    KN = [int(x) for x in (sys.argv[1:] or ["0", str(1 << 14)])]
    res = {k: ([], []) for k in KN}
    outs = {}
    for rnd in range(6):
        for k in KN:
            os.environ['DCA_TEAM_KNOBS'] = str(k)
            f, b, tf, tb = run(C, xp, whh, h0, c0, err, b4, dh, 3)
            if rnd > 0:
                res[k][0].append(tf * 1e3 / S)
                res[k][1].append(tb * 1e3 / S)
            outs[k] = [t.clone() for t in list(f) + list(b) if t is not None and t.numel() > 0]
    same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[KN[-1]]))
    for k, (f, b) in res.items():
        print(json.dumps({'knobs': k, 'fwd_us_per_step_median': float(np.median(f)),
                          'bwd_us_per_step_median': float(np.median(b)), 'fwd_min': min(f), 'bwd_min': min(b)}),
              flush=True)
    diff = max(float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))
               for a, b in zip(outs[0], outs[KN[-1]]))
    print(json.dumps({'bitwise_equal': bool(same), 'max_rel_diff': diff, 'err': int(err.item())}), flush=True)


if __name__ == '__main__':
    main()
