"""cProfile of the self-play actor runtime's host loop (VecActor.step) on one GPU: where the main thread's time goes.
Usage: python scripts/actor_cprofile.py [games] [threads] [precision] [steps]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dotaclient_amd.actor.vec import measure_vec_actor  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402

games = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 12
prec = sys.argv[3] if len(sys.argv) > 3 else 'bf16'
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 300
torch.manual_seed(0)
pol = Policy(get_config('lstm512'))
pr = cProfile.Profile()
pr.enable()
r = measure_vec_actor(pol, 'cuda', n_games=games, steps=steps, warmup=10, threads=threads, precision=prec)
pr.disable()
print(r)
pstats.Stats(pr).sort_stats('tottime').print_stats(30)
