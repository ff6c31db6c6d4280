"""Python face of the split-K TN GEMM (``csrc/gemm_tn.hip``): ``C (+)= Aᵀ·B`` for K-outer operands — the
learner's weight gradients, reduced over the B·S rows of a minibatch."""
from __future__ import annotations

from typing import Optional

import torch

from . import require

def gemm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, perm: Optional[torch.Tensor] = None,
            accumulate: bool = False, b0: Optional[torch.Tensor] = None,
            colsum: Optional[torch.Tensor] = None, exact: bool = False) -> torch.Tensor:
    """``a`` (K, M), ``b`` (K - b0_rows, N) — both bf16, or both fp32 (bf16x3 split MFMA: ≈2⁻¹⁶ relative per
    product, fp32 accumulation) — (``b0`` supplies the first rows of the B operand), result
    (M, N) f32 written to ``out`` (through row map ``perm`` if given; added to it if ``accumulate``). ``colsum``
    (M,) f32, if given, receives Σ_k a[k, m] the same way (a bias gradient, from the staged A tiles). ``exact``
    (fp32 operands): IEEE fp32 products on v_mfma_f32_16x16x4_f32 instead of the bf16x3 split."""
    C = require()
    M, N = a.shape[1], b.shape[1]
    if out is None:
        out = torch.empty(M if perm is None else int(perm.numel()), N, device=a.device, dtype=torch.float32)
    if b0 is not None and b0.shape[0] > _B0_MAX_ROWS:
        # the kernel reads b0 only in a split-K chunk's first K slab (32 rows at fp32); deeper b0: concatenate
        b, b0 = torch.cat([b0, b]), None
    C.gemm_tn(a, b, out, perm, bool(accumulate), b0, colsum, bool(exact))
    return out


_B0_MAX_ROWS = 32   # ops/csrc/gemm_tn.hip: the fp32 K slab depth (bf16: 64)
