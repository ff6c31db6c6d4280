"""Which part of the config-5 node loop trips the recurrence hand-off timeout: fp8 actor / PFSP league / 100 GB
replay, one at a time (10 s node loops, one MI355X)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dotaclient_amd.learner.e2e import measure_e2e_node  # noqa: E402

def main():
    cases = {'fp8': dict(actor_precision='fp8'), 'league': dict(league='pfsp', latest_weights_prob=0.8),
             'replay': dict(replay_gb=100.0), 'all': dict(actor_precision='fp8', league='pfsp', latest_weights_prob=0.8,
                                                          replay_gb=100.0)}
    for name in (sys.argv[1:] or list(cases)):
        try:
            r = measure_e2e_node(duration=10.0, games=2048, threads=12, precision='fp32-exact', pack=True,
                                 idle_probe=0.0, **cases[name])
            print(name, json.dumps({k: r.get(k) for k in ('steps_per_s', 'valid_steps_per_s', 'actor_steps_per_s',
                                                          'learner_gpu_ms_per_step', 'avg_weight_age')}), flush=True)
        except Exception as e:
            print(name, 'ERROR', repr(e), flush=True)


if __name__ == '__main__':
    main()
