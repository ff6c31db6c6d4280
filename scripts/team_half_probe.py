#!/usr/bin/env python3
"""Half-team probe (round 5): the exact-fp32 team recurrence with 16 CU-exclusive workgroups per XCD team
(DCA_TEAM_HALF=1) against the 32-workgroup teams, alone and with side work on a second stream.

    DCA_TEAM_HALF=0 python scripts/team_half_probe.py /tmp/half0.pt
    DCA_TEAM_HALF=1 python scripts/team_half_probe.py /tmp/half1.pt /tmp/half0.pt   # + compare

Prints one JSON line: per-step µs of the forward / backward alone, with a side GEMM load running concurrently, and
the side load's own time; with a reference file, the max relative difference of every output."""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.ops.gemm import gemm_tn  # noqa: E402
from dotaclient_amd.ops.lstm import team_ctl  # noqa: E402


def main():
    C = ops.require()
    dev = 'cuda'
    B, S, H = 8, 1400, 512
    torch.manual_seed(0)
    whh = torch.randn(4 * H, H, device=dev) * 0.04
    h0 = torch.randn(B, H, device=dev) * 0.1
    c0 = torch.randn(B, H, device=dev) * 0.1
    xp = torch.randn(S, B, H, 4, device=dev) * 0.5
    dh = torch.randn(S, B, H, device=dev) * 0.1
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    bias = torch.zeros(4 * H, device=dev)

    def fwd():
        return C.lstm_team_fwd(xp, whh, h0, c0, err, team_ctl(), True, time_major=True, bias4=bias)

    out = fwd()
    hsf, cs, gates = out[1], out[2], out[3]

    def bwd():
        return C.lstm_team_bwd(dh, gates, cs, c0, None, None, whh, err, team_ctl(), time_major=True,
                               want_dbias=True)

    bo = bwd()
    torch.cuda.synchronize()
    assert int(err.item()) == 0, f'recurrence error {int(err.item())}'
    # side load: the tail's weight-gradient GEMM shape (∂W_ih over 11 200 rows) on its own stream, repeated
    a = torch.randn(B * S, 4 * H, device=dev)
    b = torch.randn(B * S, 256, device=dev)
    side_out = torch.empty(4 * H, 256, device=dev)
    side = torch.cuda.Stream()

    def load(n):
        for _ in range(n):
            gemm_tn(a, b, out=side_out, exact=True)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    res = {}
    for name, fn in (('fwd', fwd), ('bwd', bwd)):
        fn()
        alone = min(timed(fn) for _ in range(3))
        n_load = 8
        load_alone = min(timed(lambda: load(n_load)) for _ in range(2))

        def both():
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            fn()
            with torch.cuda.stream(side):
                load(n_load)
            torch.cuda.current_stream().wait_stream(side)
        conc = min(timed(both) for _ in range(3))
        res[name] = dict(alone_us_per_step=alone / S * 1e6, load_alone_ms=load_alone * 1e3,
                         concurrent_ms=conc * 1e3, serial_ms=(alone + load_alone) * 1e3)
    torch.cuda.synchronize()
    res['err'] = int(err.item())
    outs = {'hsf': hsf, 'cs': cs, 'gates': gates, 'hn': out[4], 'cn': out[5], 'dg': bo[0], 'dh0': bo[1],
            'dc0': bo[2]}
    outs = {k: v.detach().cpu() for k, v in outs.items() if isinstance(v, torch.Tensor)}
    torch.save(outs, sys.argv[1])
    if len(sys.argv) > 2:
        ref = torch.load(sys.argv[2], weights_only=True)
        res['max_rel_diff'] = {k: float((outs[k] - ref[k]).abs().max() / ref[k].abs().max().clamp_min(1e-30))
                               for k in outs if k in ref}
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
