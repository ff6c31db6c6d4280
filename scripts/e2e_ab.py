"""End-to-end node loop on one MI355X under a few actor shapes: games per actor process × actor host threads.
Usage: python scripts/e2e_ab.py [duration] [games,threads ...]   (default 20 s; 1024,14 2048,14 2048,12)"""
import json
import sys
import time

sys.path.insert(0, '.')
from dotaclient_amd.learner.e2e import measure_e2e_node  # noqa: E402

if __name__ == '__main__':
    dur = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    shapes = [tuple(int(x) for x in a.split(',')) for a in sys.argv[2:]] or [(1024, 14), (2048, 14), (2048, 12)]
    for games, threads in shapes:
        t0 = time.time()
        r = measure_e2e_node(duration=dur, games=games, threads=threads, idle_probe=2.0,
                             progress=lambda m: print(f'[{time.time() - t0:6.1f}s] {m}', file=sys.stderr, flush=True))
        print(json.dumps({'games': games, 'threads': threads,
                          **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()
                             if not isinstance(v, (list, dict))}}), flush=True)
