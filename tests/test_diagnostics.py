"""Node-loop diagnostics added in round 5: the GIL hand-off probe (utils/gilprobe.py, DCA_GIL_PROBE), the kernel-trace
gap analysis (scripts/e2e_gaps.py) and the shared-memory capacity guard (transport/shm.py)."""
import csv
import os
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gil_probe_sees_a_gil_holder():
    import numpy as np
    from dotaclient_amd.utils.gilprobe import GilProbe
    p = GilProbe(slow_ms=2.0)

    def hog():
        a = np.random.default_rng(0).random(4_000_000)
        for _ in range(3):
            np.sort(a, kind='stable')        # holds the GIL for tens of ms per call
    th = threading.Thread(target=hog, name='hog')
    th.start()
    th.join()
    time.sleep(0.05)
    rep = p.report()
    assert p.n > 0 and len(p.late) >= 1, rep
    assert rep.startswith('[gil probe]') and 'late' in rep


def test_e2e_gaps_attributes_idle_time(tmp_path):
    """Two processes' kernel traces: the learner (runs lstm_team) busy 0-10 ms and 20-30 ms, the actor 12-15 ms —
    device busy 23 of the 30 ms window, the learner's 10 ms gap 3 ms filled by the actor."""
    def write(pid, rows):
        with open(tmp_path / f'{pid}_kernel_trace.csv', 'w', newline='') as f:
            w = csv.DictWriter(f, fieldnames=['Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
            w.writeheader()
            for n, s, e in rows:
                w.writerow({'Kernel_Name': n, 'Start_Timestamp': s, 'End_Timestamp': e})
    ms = 1_000_000
    write(100, [('lstm_team_fwd_kernel', 0, 10 * ms), ('gemm', 20 * ms, 30 * ms)])
    write(200, [('actor_core', 12 * ms, 15 * ms)])
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'e2e_gaps.py'), str(tmp_path), '--window-s',
                          '0.03'], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    txt = out.stdout
    assert 'learner pid 100' in txt
    assert 'device busy (any process): 23.0 ms' in txt, txt
    assert '10.0 ms       3.0 ms' in txt, txt       # the one learner gap (10 ms), 3 ms of it under actor kernels


def test_shm_ring_refuses_a_capacity_dev_shm_cannot_back(monkeypatch):
    import uuid
    from dotaclient_amd import native
    from dotaclient_amd.transport import shm
    if not native.AVAILABLE:
        pytest.skip('native module not built')
    monkeypatch.setattr(shm, 'shm_free_bytes', lambda: 100 << 20)
    with pytest.raises(MemoryError):
        shm.ShmBroker(f'dca_cap_{uuid.uuid4().hex[:8]}', capacity=1 << 30, create=True)
    b = shm.ShmBroker(f'dca_cap_{uuid.uuid4().hex[:8]}', capacity=16 << 20, create=True)
    b.close(unlink=True)
