"""fp8 actor encoder: wave-parallel (default) vs per-unit workgroup form, µs per call (fp16 features, 1v1 layout)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.actor.batched import fp8_weight  # noqa: E402
from dotaclient_amd.models.policy import TYPE_SUFFIX, Policy, get_config  # noqa: E402

C = ops.require()
torch.manual_seed(0)
pol = Policy(get_config('lstm512')).cuda()
U, counts = pol.config.layout.max_units, list(pol.config.layout.counts)
P = {k: v.detach().float() for k, v in pol.state_dict().items()}
wts = [fp8_weight(P[f'affine_unit_{s}.weight']) for s in TYPE_SUFFIX]
wt8 = torch.cat([q for q, _ in wts]).contiguous()
st8 = torch.stack([s_ for _, s_ in wts]).contiguous()
bt = torch.stack([P[f'affine_unit_{s}.bias'] for s in TYPE_SUFFIX]).contiguous()
w1, b1 = P['affine_unit_basic_stats.weight'].contiguous(), P['affine_unit_basic_stats.bias']
we, be = P['affine_env.weight'].contiguous(), P['affine_env.bias']
for n in (4096, 8192):
    units = torch.randn(n, U, 10, device='cuda').half()
    env = torch.randn(n, 3, device='cuda')
    outs = {}
    for per_unit in (False, True, False, True):
        f = lambda: C.encoder_fp8(units, env, w1, b1, wt8, st8, bt, we, be, counts, per_unit=per_unit)  # noqa: E731
        for _ in range(5):
            outs[per_unit] = f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f'n={n} {"per-unit" if per_unit else "wave-parallel"}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us',
              flush=True)
    same = all(torch.equal(a, b) for a, b in zip(outs[False], outs[True]))
    print(f'n={n} outputs bitwise equal: {same}', flush=True)
