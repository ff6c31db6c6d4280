"""Team-LSTM fp32 V1 at the deploy shape (B=8, S=1400, H=512): batch-major standalone call vs the learner's call
(time-major operands, folded bias, bias-gradient partials); µs per timestep, interleaved repetitions."""
import json
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from scripts.lstm_latency import _time, team_ctl  # noqa: E402


def main(B=8, S=1400, H=512, reps=5):
    C = ops.require()
    dev = 'cuda'
    torch.manual_seed(0)
    whh = torch.randn(4 * H, H, device=dev) * 0.05
    h0 = torch.zeros(B, H, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    bias = torch.randn(4 * H, device=dev) * 0.1
    xb = torch.randn(B, S, H, 4, device=dev) * 0.5
    xt = xb.transpose(0, 1).contiguous()
    dhb = torch.randn(B, S, H, device=dev)
    dht = dhb.transpose(0, 1).contiguous()
    ob = C.lstm_team_fwd(xb, whh, h0, h0, err, team_ctl(), True)
    ot = C.lstm_team_fwd(xt, whh, h0, h0, err, team_ctl(), False, None, True, None, None, None, bias)
    variants = {
        'batch_major': (lambda: C.lstm_team_fwd(xb, whh, h0, h0, err, team_ctl(), True),
                        lambda: C.lstm_team_bwd(dhb, ob[3], ob[2], h0, None, None, whh, err, team_ctl())),
        'time_major_bias': (lambda: C.lstm_team_fwd(xt, whh, h0, h0, err, team_ctl(), False, None, True, None, None,
                                                    None, bias),
                            lambda: C.lstm_team_bwd(dht, ot[3], ot[2], h0, None, None, whh, err, team_ctl(), None,
                                                    True, None, False, True)),
    }
    # learner-like neighbourhood: a big fp32 GEMM writes the input projection right before the recurrence
    a = torch.randn(S * B, 512, device=dev)
    w = torch.randn(4 * H, 512, device=dev)

    def fwd_after_gemm():
        torch.mm(a, w.t(), out=xt.view(S * B, 4 * H))
        return C.lstm_team_fwd(xt, whh, h0, h0, err, team_ctl(), False, None, True, None, None, None, bias)

    def bwd_after_gemm():
        torch.mm(a, w.t(), out=xt.view(S * B, 4 * H))
        return C.lstm_team_bwd(dht, ot[3], ot[2], h0, None, None, whh, err, team_ctl(), None, True, None, False,
                               True)
    variants['after_gemm'] = (fwd_after_gemm, bwd_after_gemm)
    gemm_only = _time(lambda: torch.mm(a, w.t(), out=xt.view(S * B, 4 * H)), reps)
    print(json.dumps({'gemm_us': gemm_only * 1e6}), flush=True)
    for rnd in range(3):
        for name, (f, b) in variants.items():
            tf, tb = _time(f, reps), _time(b, reps)
            print(json.dumps({'round': rnd, 'variant': name, 'fwd_us': tf / S * 1e6, 'bwd_us': tb / S * 1e6,
                              'err': int(err.item())}), flush=True)


if __name__ == '__main__':
    main()
