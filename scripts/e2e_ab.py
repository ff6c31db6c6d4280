"""End-to-end node loop on one MI355X under a few actor shapes: games per actor process × actor host threads
[× actor policy precision bf16 | fp8]; the learner as in bench.py (fp32-exact, packed sequences).
Usage: python scripts/e2e_ab.py [duration] [games,threads[,precision[,actor_procs]] ...]
(default 20 s; 1024,14 2048,14 2048,12)"""
import json
import sys
import time

sys.path.insert(0, '.')
from dotaclient_amd.learner.e2e import measure_e2e_node  # noqa: E402

if __name__ == '__main__':
    dur = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    shapes = [(a.split(',') + ['bf16', '1'][len(a.split(',')) - 2:])[:4] for a in sys.argv[2:]] or \
        [('1024', '14', 'bf16', '1'), ('2048', '14', 'bf16', '1'), ('2048', '12', 'bf16', '1')]
    for games, threads, prec, procs in shapes:
        games, threads, procs = int(games), int(threads), int(procs)
        t0 = time.time()
        r = measure_e2e_node(duration=dur, games=games, threads=threads, idle_probe=2.0, precision='fp32-exact',
                             pack=True, actor_precision=prec, actor_procs=procs,
                             progress=lambda m: print(f'[{time.time() - t0:6.1f}s] {m}', file=sys.stderr, flush=True))
        print(json.dumps({'games': games, 'threads': threads, 'actor_precision': prec, 'actor_procs': procs,
                          **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()
                             if not isinstance(v, (list, dict))}}), flush=True)
