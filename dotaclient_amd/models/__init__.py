"""Policy models: torch reference (``policy``) and the fused MI355X path (``fused``)."""
from .policy import (Policy, PolicyConfig, PRESETS, get_config, masked_log_softmax, batched_action_masks,  # noqa
                     RndModel, EntityAttention)
