"""Host-side sanitizers (SURVEY §5 race detection / sanitizers): the native decoder + featurizer is fuzzed and the
shared-memory ring is driven by concurrent producers/consumers under ASan+UBSan and under TSan
(dotaclient_amd/native/sanitize_main.cpp over core.h). CPU only; GPU sanitizers are not available on this pool."""
import os
import struct
import subprocess

import pytest

from dotaclient_amd.native.build import build_sanitizer


def _seed_file(path):
    from tests.test_native import _states
    from dotaclient_amd.env import get_1v1_selfplay_config, get_5v5_selfplay_config
    n = 0
    with open(path, 'wb') as f:
        for cfg in (get_1v1_selfplay_config, get_5v5_selfplay_config):
            for s in _states(cfg, n_steps=60, seed=3):
                b = s if isinstance(s, bytes) else s[0]
                f.write(struct.pack('<I', len(b)) + b)
                n += 1
    return n


@pytest.mark.parametrize('kind', ['asan', 'tsan'])
def test_native_core_under_sanitizer(tmp_path, kind):
    try:
        exe = build_sanitizer(kind)
    except (subprocess.CalledProcessError, FileNotFoundError) as e:   # toolchain without the runtime
        pytest.skip(f'cannot build {kind} driver: {e}')
    seeds = str(tmp_path / 'seeds.bin')
    assert _seed_file(seeds) > 0
    env = dict(os.environ, ASAN_OPTIONS='verify_asan_link_order=0:detect_leaks=1',
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1', TSAN_OPTIONS='halt_on_error=1')
    out = subprocess.run([exe, seeds, '4000' if kind == 'tsan' else '20000'], env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-4000:])
    assert 'all sanitizer checks passed' in out.stdout
