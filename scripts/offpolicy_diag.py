#!/usr/bin/env python3
"""GPU diagnostic of the learner-side policy_old pass (learner/optimizer.py old_logp='learner'): rollouts from the
IEEE-fp32 actor at version-0 weights → the optimizer's device ingest (packed sequences) at the SAME weights: the
learner's log-probs must equal the actor's (behaviour KL ≈ 0, ρ ≈ 1); the first minibatch's PPO ratio is exactly 1
(approx_kl 0, clipfrac 0); then per-minibatch KL of a few steps, and the same with the bf16 actor."""
import json
import sys
import time

import torch

sys.path.insert(0, '.')


def main(precision='fp32', steps=6, pack=True):
    from dotaclient_amd.actor.vec import VecActor
    from dotaclient_amd.actor.weights import WeightStore
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.models.policy import Policy
    from dotaclient_amd.transport.broker import InProcBroker
    from dotaclient_amd.transport.codec import decode
    torch.manual_seed(3)
    pol = Policy('lstm512')
    ws = WeightStore('lstm512', device='cpu')
    ws.add(0, {k: v.detach().clone() for k, v in pol.state_dict().items()})
    sent = []
    va = VecActor(ws, 256, sent.append, device='cuda', seed=5, rollout_size=9999, max_dota_time=600.0,
                  hidden_stride=1400, threads=8, stagger=True, precision=precision)
    t0 = time.time()
    total, seen = 0, 0
    while time.time() - t0 < 180 and total < 26 * 1400:
        va.step()
        for b in sent[seen:]:
            total += decode(b).length
        seen = len(sent)
    va.close()
    rs = [decode(b) for b in sent]
    cfg = OptimizerConfig(log_dir='/tmp/dca_offdiag', batch_size=8, seq_len=1400, seq_per_epoch=16, epochs=1,
                          model='lstm512', device='cuda', ingest='device', old_logp='learner', pack_sequences=pack)
    opt = DotaOptimizer(cfg, InProcBroker())
    opt.policy.load_state_dict(ws.latest_weights()[1])
    opt.learner.after_load_weights()
    st = opt._ingest_pipeline(thread=False).stage(rs)
    n = min(16, st.n_seq - st.n_seq % 8)
    assert n >= 16, (st.n_seq, len(rs))
    d = opt._finish_ingest(st, n)
    use = rs
    prox = {k: float(v) for k, v in d.pop('_prox').items()}
    out = {'actor_precision': precision, 'rollouts': len(use), 'prox': prox}
    pool = opt._iteration_pool(d, 16)
    kls = []
    for s in range(steps):
        idx = torch.arange(8 * (s % 2), 8 * (s % 2) + 8, device='cuda')
        m = opt.learner.train_step_indices(pool, idx)
        kls.append({k: float(m[k]) for k in ('approx_kl', 'clipfrac', 'grad_norm', 'entropy', 'loss')})
    torch.cuda.synchronize()
    opt.learner.check_error()
    out['steps'] = kls
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main('fp32')
    main('bf16')
