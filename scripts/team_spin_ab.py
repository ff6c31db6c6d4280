"""A/B of the team-LSTM poll back-off (DCA_TEAM_KNOBS bits 12/13) on the fp32 V1 path at the deploy shape
(B=8, S=1400, H=512): µs per timestep forward and backward, interleaved repetitions."""
import json
import os
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from scripts.lstm_latency import _time, team_ctl  # noqa: E402


def run(B=8, S=1400, H=512, reps=5):
    C = ops.require()
    dev = 'cuda'
    torch.manual_seed(0)
    whh = torch.randn(4 * H, H, device=dev) * 0.05
    h0 = torch.zeros(B, H, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    dh = torch.randn(B, S, H, device=dev)
    xp = torch.randn(B, S, H, 4, device=dev) * 0.5
    out = C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), True)
    res = {}
    for rnd in range(3):
        for k in [int(a) for a in (sys.argv[1:] or ['0', '4096', '8192', '12288'])]:
            os.environ['DCA_TEAM_KNOBS'] = str(k)
            tf = _time(lambda: C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), True), reps)
            tb = _time(lambda: C.lstm_team_bwd(dh, out[3], out[2], h0, None, None, whh, err, team_ctl()), reps)
            res.setdefault(k, []).append((tf / S * 1e6, tb / S * 1e6))
            print(json.dumps({'round': rnd, 'knobs': k, 'fwd_us': tf / S * 1e6, 'bwd_us': tb / S * 1e6,
                              'err': int(err.item())}), flush=True)
    for k, v in res.items():
        print(json.dumps({'knobs': k, 'fwd_min': min(a for a, _ in v), 'bwd_min': min(b for _, b in v)}))


if __name__ == '__main__':
    run()
