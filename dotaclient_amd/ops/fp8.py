"""FP8 (OCP e4m3) GEMMs for policy inference on MI355X (BASELINE.json config 5: "fp8 MFMA policy GEMMs").

CDNA4 runs e4m3 MFMA at twice the bf16 rate. The policy's plain GEMMs (pre-RNN 896→H, the LSTM input/recurrent
projections, the fused heads) go through hipBLASLt's fp8 path (``torch._scaled_mm``) with

* weights: per-tensor scale ``amax/448`` computed once per weight load (static, like any inference engine);
* activations: per-tensor scale computed ON DEVICE every call (``amax`` reduction → scale tensor), so the whole
  step stays hipGraph-capturable and no host sync is needed;
* fp32 accumulation; output in fp32 (``out_dtype``) so the fused sampling / LSTM-cell kernels see full-precision
  pre-activations.

The learner keeps bf16 (the headline benchmark dtype); fp8 is an actor-side option (``GpuActorPolicy(fp8=True)``,
``cli.agent --fp8``).
"""
from __future__ import annotations

import torch

E4M3 = torch.float8_e4m3fn
E4M3_MAX = 448.0


def quantize(t: torch.Tensor, scale: torch.Tensor = None):
    """Per-tensor e4m3 quantisation; returns (q, scale) with t ≈ q.float() * scale. ``scale`` is a 0-dim fp32
    device tensor (computed from the amax when not given)."""
    if scale is None:
        scale = (t.detach().abs().amax().float() / E4M3_MAX).clamp_min(1e-12)
    q = (t.float() / scale).clamp(-E4M3_MAX, E4M3_MAX).to(E4M3)
    return q, scale


class Fp8Weight:
    """A weight ``W (N, K)`` kept as e4m3 ``Wᵀ`` (column-major view for ``_scaled_mm``) + its scale."""

    def __init__(self, w: torch.Tensor):
        q, s = quantize(w)
        self.qt = q.t()              # (K, N) column-major — the layout hipBLASLt's fp8 path wants for operand B
        self.scale = s
        self.shape = tuple(w.shape)

    def load_(self, w: torch.Tensor):
        """In-place reload (keeps addresses stable for captured graphs)."""
        q, s = quantize(w)
        self.qt.copy_(q.t())
        self.scale.copy_(s)


def linear(x: torch.Tensor, w: Fp8Weight, bias: torch.Tensor = None, out_dtype=torch.float32) -> torch.Tensor:
    """``x (M, K) → x·Wᵀ (+ bias)`` on the fp8 MFMA path with a dynamic per-tensor activation scale."""
    xq, xs = quantize(x)
    y = torch._scaled_mm(xq, w.qt, scale_a=xs, scale_b=w.scale, out_dtype=out_dtype)
    return y + bias if bias is not None else y
