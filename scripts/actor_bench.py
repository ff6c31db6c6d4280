"""Batched GPU actor throughput alone (for rocprofv3): python3 scripts/actor_bench.py [n_games] [bf16|fp32|fp8]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dotaclient_amd.actor.batched import measure_actor_throughput  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

n_games = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
torch.manual_seed(0)
policy = Policy(get_config('lstm512'))
prec = sys.argv[2] if len(sys.argv) > 2 else 'bf16'
print(json.dumps(measure_actor_throughput(policy, torch.device('cuda:0'), n_games=n_games, precision=prec)))
