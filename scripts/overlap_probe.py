#!/usr/bin/env python3
"""Does concurrent work on a second stream slow the persistent LSTM recurrence?  The team kernels occupy one
workgroup per CU and are latency-bound, so the rest of each CU is idle; this probe times lstm_team_fwd/bwd (B=8,
S=1400, H=512) alone and with a stream of bandwidth-heavy (GEMM / copy) work running next to it."""
import json
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.ops.lstm import team_ctl  # noqa: E402


def main():
    C = ops.require()
    dev = 'cuda'
    B, S, H = 8, 1400, 512
    torch.manual_seed(0)
    f32 = 'f32' in sys.argv          # the fp32 learner's recurrence (exact-fp32 VALU V1 forward / V2 backward)
    whh = torch.randn(4 * H, H, device=dev) * 0.05
    if not f32:
        whh = whh.to(torch.bfloat16)
    h0 = torch.zeros(B, H, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    dh = torch.randn(B, S, H, device=dev)
    xp = torch.randn(B, S, H, 4, device=dev) * 0.5
    out = C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), not f32)
    fwd = lambda: C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), not f32)  # noqa: E731
    bwd = lambda: C.lstm_team_bwd(dh, out[3], out[2], h0, None, None, whh, err, team_ctl())  # noqa: E731
    a = torch.randn(89600, 512, device=dev).to(torch.bfloat16)
    w = torch.randn(512, 2048, device=dev).to(torch.bfloat16)
    big = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    big2 = torch.empty_like(big)
    from dotaclient_amd.ops.gemm import gemm_tn
    dg = torch.randn(11200, 2048, device=dev)
    hs = torch.randn(11200, 512, device=dev)
    loads = {
        'none': None,
        'gemm_tn_f32': lambda: gemm_tn(dg, hs),
        'gemm': lambda: torch.mm(a, w),
        'copy': lambda: big2.copy_(big),
        'small_gemm': lambda: torch.mm(a[:11200], w),
    }
    side = torch.cuda.Stream()
    res = {}
    for name, fn in (('fwd', fwd), ('bwd', bwd)):
        for lname, load in loads.items():
            fn()
            torch.cuda.synchronize()
            # time one load call alone
            t_load = None
            if load is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                load()
                torch.cuda.synchronize()
                e0.record()
                for _ in range(10):
                    load()
                e1.record()
                torch.cuda.synchronize()
                t_load = e0.elapsed_time(e1) / 10
            ts, tser = [], []
            n = 0 if load is None else max(1, int(round(0.6 / t_load)))   # ~0.6 ms of side work
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                side.wait_stream(torch.cuda.current_stream())
                if load is not None:
                    with torch.cuda.stream(side):
                        for _ in range(n):
                            load()
                fn()
                torch.cuda.current_stream().wait_stream(side)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
                e0.record()
                fn()
                for _ in range(n):
                    load() if load is not None else None
                e1.record()
                torch.cuda.synchronize()
                tser.append(e0.elapsed_time(e1))
            res[f'{name}/{lname}'] = {'concurrent_ms': min(ts), 'serial_ms': min(tser), 'n': n, 'load_ms_alone': t_load}
            print(json.dumps({f'{name}/{lname}': res[f'{name}/{lname}']}), flush=True)
    print('err', int(err.item()))


if __name__ == '__main__':
    main()
