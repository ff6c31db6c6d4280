"""fp32-exact learner vs float64 at the deploy shape, per loss algorithm: which tensors are furthest off.
python scripts/exact_diag.py [algo ...]   (default: ppo vpg)"""
import sys

sys.path.insert(0, '.')
from tests.test_fp32_kernels import _rel, _step_grads  # noqa: E402

for algo in sys.argv[1:] or ['ppo', 'vpg']:
    (lf, _, gf), (lo, _, go), (l64, g64) = _step_grads('fp32-exact', 'lstm512', algo, 8, 1400, fp64=True)
    rows = sorted(((_rel(gf[n], g64[n]), _rel(go[n], g64[n]), n) for n in g64
                   if g64[n] is not None and g64[n].norm() > 0), reverse=True)
    print(algo, 'loss', lf, lo, l64, flush=True)
    for r in rows[:8]:
        print(f'  {r[2]:40s} fused {r[0]:.3e}  torch-fp32 {r[1]:.3e}', flush=True)
