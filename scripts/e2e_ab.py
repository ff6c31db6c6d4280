"""End-to-end loop on one MI355X: actor as a thread (in-process queues) vs actor as a process (shm broker)."""
import json
import sys

sys.path.insert(0, '.')
from dotaclient_amd.learner.e2e import measure_e2e, measure_e2e_procs  # noqa: E402

if __name__ == '__main__':
    for name, fn in (('process', measure_e2e_procs), ('thread', measure_e2e)):
        r = fn(duration=20.0)
        print(json.dumps({'mode': name, **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}}),
              flush=True)
