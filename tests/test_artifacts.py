"""Artifact store (reference GCS upload / resume / --model download): local + fsspec backends, background uploads,
optimizer mirroring and resume from the store, DP optimizer-state broadcast on resume."""
import os

import numpy as np
import pytest
import torch

from dotaclient_amd.utils import artifacts as art


@pytest.mark.parametrize('kind', ['local', 'memory'])
def test_store_put_get_list(tmp_path, kind):
    url = str(tmp_path / 'store') if kind == 'local' else 'memory://dca-test-store'
    st = art.open_store(url)
    src = tmp_path / 'a.bin'
    src.write_bytes(b'xyz' * 100)
    st.put(str(src), 'run1/model_000000003.pt')
    st.put(str(src), 'run1/model_000000010.pt')
    assert st.list('run1') == ['run1/model_000000003.pt', 'run1/model_000000010.pt']
    assert st.exists('run1/model_000000010.pt') and not st.exists('run1/nope.pt')
    dst = tmp_path / 'out' / 'b.bin'
    st.get('run1/model_000000010.pt', str(dst))
    assert dst.read_bytes() == b'xyz' * 100


def test_missing_backend_fails_loudly():
    with pytest.raises(RuntimeError):
        art.open_store('nosuchproto://bucket/x')


def test_resolve_model_path(tmp_path):
    st = art.open_store(str(tmp_path / 's'))
    f = tmp_path / 'm.pt'
    torch.save({'w': torch.ones(2)}, f)
    st.put(str(f), 'exp/model_000000001.pt')
    local = art.resolve_model_path(f'file://{tmp_path / "s"}#exp/model_000000001.pt', cache_dir=str(tmp_path / 'c'))
    assert torch.load(local, weights_only=True)['w'].sum() == 2
    assert art.resolve_model_path(str(f)) == str(f)


def test_optimizer_mirrors_and_resumes_from_store(tmp_path):
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.transport.broker import InProcBroker
    from dotaclient_amd.transport.codec import encode
    from tests.test_returns_scan import _rollouts
    store = str(tmp_path / 'bucket')
    log_dir = str(tmp_path / 'run' / 'exp1')

    def make(ld):
        cfg = OptimizerConfig(log_dir=ld, batch_size=2, seq_len=32, seq_per_epoch=4, epochs=1, model='lstm128',
                              device='cpu', backend='torch', run_local=False, artifact_url=store)
        return DotaOptimizer(cfg, InProcBroker())
    opt = make(log_dir)
    for r in _rollouts(6, H=opt.policy_cfg.hidden):
        opt.broker.publish_experience(encode(r))
    opt.run(iterations=2)
    keys = art.open_store(store).list('exp1')
    assert 'exp1/model_000000002.pt' in keys and 'exp1/trainer_state_000000002.pt' in keys
    assert any(os.path.basename(k).startswith('events.out.tfevents') for k in keys)
    # a fresh node (empty local dir, same run name) resumes from the store
    opt2 = make(str(tmp_path / 'other_node' / 'exp1'))
    assert opt2.iteration_start == 3
    for (n1, p1), (n2, p2) in zip(opt.policy.named_parameters(), opt2.policy.named_parameters()):
        assert torch.equal(p1.detach().cpu(), p2.detach().cpu()), n1
    np.testing.assert_array_equal(opt2.learner.opt.exp_avg.numpy(), opt.learner.opt.exp_avg.numpy())
