"""Run presets (dotaclient_amd/presets.py): every BASELINE config maps onto each entrypoint's flags."""
import json

import pytest

from dotaclient_amd.presets import PRESETS, parse_with_preset


def _parsers():
    import importlib
    out = {}
    for role, mod in (('optimizer', 'dotaclient_amd.cli.optimizer'), ('agent', 'dotaclient_amd.cli.agent'),
                      ('launch', 'dotaclient_amd.cli.launch')):
        out[role] = importlib.import_module(mod).build_parser
    return out


def test_five_presets_cover_baseline_configs():
    cfgs = json.load(open('BASELINE.json'))['configs']
    assert len(PRESETS) == len(cfgs) == 5
    assert sorted(p.world_size for p in PRESETS.values()) == [1, 1, 1, 8, 8]


@pytest.mark.parametrize('name', sorted(PRESETS))
def test_preset_sets_role_defaults_and_flags_win(name):
    p = PRESETS[name]
    for role, build in _parsers().items():
        args = parse_with_preset(build(), role, ['--preset', name])
        for k, v in getattr(p, role).items():
            assert getattr(args, k) == v, (role, k)
    # an explicit flag overrides the preset
    args = parse_with_preset(_parsers()['optimizer'](), 'optimizer', ['--preset', name, '--batch-size', '3'])
    assert args.batch_size == 3


def test_bench_parser_accepts_presets(monkeypatch):
    import sys
    sys.path.insert(0, '.')
    import bench
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--preset', 'cpu-plumbing'])
    a = bench.parse()
    assert (a.model, a.batch_size, a.seq_len) == ('lstm128', 4, 256)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--preset', 'lstm512-8gpu', '--steps', '3'])
    a = bench.parse()
    assert (a.model, a.batch_size, a.seq_len, a.steps, a.precision) == ('lstm512', 8, 1400, 3, 'fp32-exact')
