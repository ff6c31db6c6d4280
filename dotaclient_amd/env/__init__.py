"""Environment: synthetic DotaService, game configs, gRPC transport for the DotaService contract."""
from .synthetic import SyntheticDotaService, SyntheticGame  # noqa: F401
from .configs import get_1v1_selfplay_config, get_1v1_bot_vs_default_config, get_5v5_selfplay_config  # noqa: F401
