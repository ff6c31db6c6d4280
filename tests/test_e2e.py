"""End-to-end loop (learner/e2e.py) on CPU: VecActor thread → bounded queue → DotaOptimizer → model broadcast."""
import os
import pytest

from dotaclient_amd import native

pytestmark = pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')


def test_e2e_actor_learner_loop_cpu():
    from dotaclient_amd.learner.e2e import measure_e2e
    r = measure_e2e(model='lstm128', device='cpu', duration=60.0, max_iterations=4, games=8, threads=2, seq_len=64,
                    batch_size=4, seq_per_epoch=8, max_dota_time=20.0, warmup_iterations=1)
    assert r['iterations'] == 4
    assert r['steps_per_s'] > 0 and 0 < r['valid_steps_per_s'] <= r['steps_per_s']
    # models flow back to the actor: rollouts are at most a few versions old
    assert 0 <= r['avg_weight_age'] < 4
    assert r['actor_steps_per_s'] > 0


def test_e2e_actor_process_over_shm_cpu():
    """The deploy's process split: VecActor in a spawned process, rollouts and models through the shared-memory
    broker (native ring + model slot), the learner here."""
    import glob
    from dotaclient_amd.learner.e2e import measure_e2e_procs
    mine = f'/dev/shm/dca_e2e_{os.getpid()}_*'
    r = measure_e2e_procs(model='lstm128', device='cpu', duration=180.0, max_iterations=3, games=8, threads=2,
                          seq_len=64, batch_size=4, seq_per_epoch=8, max_dota_time=20.0, warmup_iterations=1)
    assert r['iterations'] == 3
    assert r['steps_per_s'] > 0 and r['actor_steps_per_s'] > 0
    assert 0 <= r['avg_weight_age'] < 8
    assert glob.glob(mine) == []                                   # ring and model slot unlinked
