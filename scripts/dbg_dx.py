import torch, sys
sys.path.insert(0, '.')
from dotaclient_amd import ops
C = ops.require()
torch.manual_seed(0)

def report(name, got, ref):
    err = (got.double() - ref).abs()
    print(name, 'rel max err', (err.max() / ref.abs().max()).item(), flush=True)
    rows_bad = (err.max(1).values > 1e-3 * ref.abs().max()).nonzero().flatten().tolist()
    cols_bad = (err.max(0).values > 1e-3 * ref.abs().max()).nonzero().flatten().tolist()
    print('  bad rows', len(rows_bad), rows_bad[:40]); print('  bad cols', len(cols_bad), cols_bad[:40])

for N in (48, 96, 1000):
    K = 512
    A = torch.randn(N, K, device='cuda')
    W = torch.randn(256, K, device='cuda') * 0.05
    b = torch.randn(256, device='cuda')
    nil = W.new_empty(0)
    report(f'N={N} out256 exact', C.rowmm_out256(A, W, nil, b), A.double() @ W.double().t() + b.double())
    report(f'N={N} out256 bf16x3', C.rowmm_out256(A, *C.split_bf16x2(W, True), b), A.double() @ W.double().t() + b.double())
    dz = torch.randn(N, 256, device='cuda')
    report(f'N={N} in256 exact', C.rowmm_in256(dz, W.t().contiguous(), nil), dz.double() @ W.double())
    K1, P, X = 2048, 256, 896
    dG = torch.randn(N, K1, device='cuda') * 1e-3
    wihT = torch.randn(P, K1, device='cuda') * 0.05
    x = torch.relu(torch.randn(N, P, device='cuda'))
    wpreT = torch.randn(X, P, device='cuda') * 0.05
    e = wihT.new_empty(0)
    dpre, dx = C.dpre_dx(dG, wihT, e, x, wpreT, e)
    ref_pre = (dG.double() @ wihT.double().t()) * (x > 0)
    report(f'N={N} dpre exact', dpre, ref_pre)
    report(f'N={N} dx exact', dx, ref_pre @ wpreT.double().t())
