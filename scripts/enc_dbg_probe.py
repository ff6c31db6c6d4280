"""Exact encoder forward under DCA_ENC_DBG knobs (each run in its own process): which phase costs what."""
import os
import subprocess
import sys

code = r'''
import torch, sys
sys.path.insert(0, '.')
from dotaclient_amd import ops
C = ops.require()
N, U = 11200, 40
g = torch.Generator(device='cuda').manual_seed(0)
r = lambda *s: torch.randn(*s, device='cuda', generator=g)
units, env = r(N, U, 10), r(N, 3)
w1, b1, wt, bt, we, be = r(128, 10) * 0.3, r(128) * 0.1, r(6, 128, 128) * 0.1, r(6, 128) * 0.1, r(128, 3), r(128)
f = lambda: C.encoder_fwd(units, env, w1, b1, wt, bt, we, be, [1, 5, 16, 16, 1, 1], False, exact=True)
for _ in range(3): f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): f()
e1.record(); torch.cuda.synchronize()
print(f"{e0.elapsed_time(e1) * 1e3 / 20:.1f}")
'''
for dbg in [0, 1, 2, 4, 8, 3, 7, 15]:
    env = dict(os.environ, DCA_ENC_DBG=str(dbg))
    out = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=300)
    print(f'DCA_ENC_DBG={dbg:2d}: {out.stdout.strip()} us {out.stderr.strip()[-200:] if out.returncode else ""}',
          flush=True)
