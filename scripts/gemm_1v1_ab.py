"""1v1 learner GEMM shapes (B·S = 11 200 rows, fast fp32): bias/activation epilogues vs plain GEMM + elementwise."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


torch.backends.cuda.matmul.allow_tf32 = True
cfg = get_config('lstm512')
pol = Policy(cfg)
wpre = pol.affine_pre_rnn.weight.detach().cuda()
bpre = pol.affine_pre_rnn.bias.detach().cuda()
R = 11200
x896 = torch.randn(R, wpre.shape[1], device='cuda')
wh = torch.randn(160, cfg.hidden, device='cuda')
bh = torch.randn(160, device='cuda')
hs = torch.randn(R, cfg.hidden, device='cuda')
res = {'pre_shape': list(wpre.shape)}
res['pre_addmm_relu'] = t(lambda: torch._addmm_activation(bpre, x896, wpre.t()))
res['pre_addmm'] = t(lambda: torch.addmm(bpre, x896, wpre.t()))
res['pre_mm'] = t(lambda: torch.mm(x896, wpre.t()))
res['pre_mm_bias_relu'] = t(lambda: torch.relu_(torch.mm(x896, wpre.t()).add_(bpre)))
wpreT = wpre.t().contiguous()
res['pre_mm_Kcontig'] = t(lambda: torch.mm(x896, wpreT))
res['heads_addmm'] = t(lambda: torch.addmm(bh, hs, wh.t()))
res['heads_mm'] = t(lambda: torch.mm(hs, wh.t()))
res['heads_mm_bias'] = t(lambda: torch.mm(hs, wh.t()).add_(bh))
print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}))
