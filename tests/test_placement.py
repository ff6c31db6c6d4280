"""Host placement of a node's ranks (parallel/placement.py): GPU-local NUMA shares, even splits, cgroup quota
capping of the thread budget — the reference's per-pod CPU sizing (ks-app/components/agent.jsonnet:45-49,
optimizer.jsonnet:143-148) made explicit for 8 ranks + 8 actor processes on one node."""
import os

from dotaclient_amd.parallel import placement as P


def test_cpulist_roundtrip():
    assert P.parse_cpulist('0-3,8,10-11') == [0, 1, 2, 3, 8, 10, 11]
    assert P.cpulist_str([0, 1, 2, 3, 8, 10, 11]) == '0-3,8,10-11'
    assert P.parse_cpulist(P.cpulist_str(range(5, 70))) == list(range(5, 70))


def test_numa_shares_are_disjoint_and_gpu_local():
    nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    node_cpus = {0: list(range(0, 64)) + list(range(128, 192)), 1: list(range(64, 128)) + list(range(192, 256))}
    plans = [P.plan(r, 8, affinity=range(256), quota=None, gpu_nodes=nodes, node_cpus=node_cpus) for r in range(8)]
    seen = set()
    for r, p in enumerate(plans):
        assert p.source == 'numa' and p.numa_node == nodes[r]
        assert set(p.cpus) <= set(node_cpus[nodes[r]])          # every CPU of the share is local to the rank's GPU
        assert not (seen & set(p.cpus))                          # no two ranks share a CPU
        seen |= set(p.cpus)
        assert len(p.cpus) == 32 and p.share == 32
        assert p.threads(reserve=2) == 30


def test_quota_caps_the_thread_budget_not_the_mask():
    # one GPU on a big machine whose container gets 16 CPUs of quota: the mask is the GPU's NUMA node, the thread
    # budget is the quota
    p = P.plan(0, 1, affinity=range(256), quota=16, gpu_nodes=[1], node_cpus={1: range(64, 128)})
    assert p.source == 'numa' and p.cpus == list(range(64, 128)) and p.share == 16
    assert min(14, p.threads(reserve=2)) == 14


def test_eight_rank_thread_sizing_under_quota():
    """The thread counts bench.py / the node loop use for 8 ranks: a 16-CPU quota leaves 1 actor thread per rank
    (the learner keeps the other CPU of its 2-CPU share), a 128-CPU quota the 14-thread cap."""
    nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    node_cpus = {0: list(range(0, 64)) + list(range(128, 192)), 1: list(range(64, 128)) + list(range(192, 256))}
    for quota, expect in ((16, 1), (128, 14), (32, 3), (8, 1)):
        plans = [P.plan(r, 8, affinity=range(256), quota=quota, gpu_nodes=nodes, node_cpus=node_cpus)
                 for r in range(8)]
        assert all(p.share == max(1, quota // 8) for p in plans)
        assert [p.actor_threads() for p in plans] == [expect] * 8
        # the node's actor threads plus one learner CPU per rank never exceed the quota once it is ≥ 2 per rank
        if quota >= 16:
            assert sum(p.actor_threads() + 1 for p in plans) <= quota
    # one rank with the whole 16-CPU box share: the measured 14-thread point
    p = P.plan(0, 1, affinity=range(256), quota=16, gpu_nodes=[0], node_cpus=node_cpus)
    assert p.actor_threads() == 14


def test_even_split_without_topology():
    plans = [P.plan(r, 4, affinity=range(8), quota=None, gpu_nodes=None, node_cpus={}) for r in range(4)]
    assert all(p.source == 'even-split' for p in plans)
    assert [p.cpus for p in plans] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    # more ranks than CPUs: every rank keeps the whole mask
    p = P.plan(5, 16, affinity=range(8), quota=None, gpu_nodes=None, node_cpus={})
    assert p.source == 'affinity' and p.cpus == list(range(8))


def test_cgroup_quota_parse(tmp_path):
    (tmp_path / 'cpu.max').write_text('1600000 100000\n')
    assert P.cgroup_cpu_quota(str(tmp_path)) == 16
    (tmp_path / 'cpu.max').write_text('max 100000\n')
    assert P.cgroup_cpu_quota(str(tmp_path)) is None


def test_apply_pins_the_calling_thread():
    before = os.sched_getaffinity(0)
    try:
        p = P.Placement(0, 1, sorted(before)[:1])
        assert P.apply(p)
        assert os.sched_getaffinity(0) == set(p.cpus)
    finally:
        os.sched_setaffinity(0, before)
