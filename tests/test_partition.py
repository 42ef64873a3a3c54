"""Partitioned mode (BASELINE config #5): the multi-rank exchange
protocol of keto_amd.partition.PartitionedEngine against the oracle.

CPU tests run the protocol for real over gloo with world_size 2 and 3, with each rank's
device steps played by tests/part_cpu.py; the GPU tests run the HIP steps
(partition.hip) with world_size 1 and with two ranks sharing the box's GPU over gloo."""
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from keto_amd import _lib as L
from keto_amd import relationtuple as rt
from keto_amd.snapshot import Snapshot
from tests import randgraph
from tests.part_cpu import owner


def _case(seed, n_rows=900, n_req=700):
    namespaces, rows = randgraph.make_graph(seed, n_rows=n_rows, n_obj=40, n_users=60, poison=True)
    reqs = randgraph.make_requests(seed, namespaces, rows, n=n_req, wildcard=False)
    return namespaces, rows, reqs


def _ids(snap, reqs):
    return snap.resolve_many([(ns, o, r, rt.subject_from_dict(s)) for ns, o, r, s in reqs])


def _want(namespaces, rows, reqs):
    return randgraph.oracle_store(namespaces, rows).check_batch(reqs).astype(bool)


def test_owner_matches_library():
    lib = L.lib()
    vs = np.array([0, 1, 2, 3, 1000, 123456, 0x7FFFFFFF, 0xFFFFFFFE], dtype=np.uint64)
    for world in (1, 2, 3, 8, 64):
        assert owner(vs, world).tolist() == [lib.ketogpu_part_owner(int(v), world) for v in vs]


@pytest.mark.parametrize("direction", ["forward", "backward", "auto"])
def test_protocol_single_rank_cpu(direction):
    from keto_amd.partition import PartitionedEngine
    from tests.part_cpu import CpuPartition
    namespaces, rows, reqs = _case(61)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    roots, targets = _ids(snap, reqs)
    eng = PartitionedEngine(snap, local=CpuPartition(snap.graph(), 0, 1, words=3), direction=direction)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), _want(namespaces, rows, reqs))
    if direction == "auto":  # both directions ran a trial round, then one was kept
        assert set(eng._trial) == {0, 1} and eng.direction in (0, 1)


def _worker(rank, world, port, seed, out_dir, device_steps, direction="auto"):
    import torch.distributed as dist
    from keto_amd.partition import PartitionedEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        namespaces, rows, reqs = _case(seed)
        snap = Snapshot.from_rows(namespaces, rows, sort=True)
        roots, targets = _ids(snap, reqs)
        if device_steps:
            eng = PartitionedEngine(snap, device=0, record_capacity=4096, max_words_per_round=4, direction=direction)
        else:
            from tests.part_cpu import CpuPartition
            eng = PartitionedEngine(snap, local=CpuPartition(snap.graph(), rank, world, words=4), direction=direction)
        got = eng.check_ids(roots, targets)
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), got)
        np.save(os.path.join(out_dir, f"records{rank}.npy"), np.array([eng.records, eng.levels]))
        eng.close()
    finally:
        dist.destroy_process_group()


def _run_ranks(world, seed, device_steps, port, direction="auto"):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, port, seed, d, device_steps, direction), nprocs=world, join=True,
                           start_method="spawn")
        got = [np.load(os.path.join(d, f"rank{r}.npy")) for r in range(world)]
        rec = [np.load(os.path.join(d, f"records{r}.npy")) for r in range(world)]
    return got, rec


@pytest.mark.parametrize("world,seed,direction", [(2, 62, "forward"), (2, 62, "backward"), (3, 63, "auto")])
def test_protocol_multi_rank_gloo(world, seed, direction):
    namespaces, rows, reqs = _case(seed)
    want = _want(namespaces, rows, reqs)
    port = 29600 + world + 10 * ["forward", "backward", "auto"].index(direction)
    got, rec = _run_ranks(world, seed, device_steps=False, port=port, direction=direction)
    for g in got:  # every rank returns the full answer
        np.testing.assert_array_equal(g, want)
    assert all(r[0] > 0 for r in rec)  # records really crossed ranks
    assert want.any() and not want.all()


# --------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("direction", ["forward", "backward"])
@pytest.mark.parametrize("seed", [71, 72])
def test_partition_device_single_rank(seed, direction):
    from keto_amd.partition import PartitionedEngine
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows, reqs = _case(seed, n_rows=1500, n_req=3000)
    snap = Snapshot.from_rows(namespaces, rows, sort=True)
    roots, targets = _ids(snap, reqs)
    want = _want(namespaces, rows, reqs)
    eng = PartitionedEngine(snap, device=0, max_words_per_round=8, direction=direction)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    st = eng.local.stats()
    assert st["rounds"] >= 6 and st["levels"] > 0 and st["records_sent"] > 0
    # tiny buffers: rounds overflow and are retried with fewer words, same answers
    small = PartitionedEngine(snap, device=0, record_capacity=2048, max_words_per_round=8, direction=direction)
    np.testing.assert_array_equal(small.check_ids(roots, targets), want)
    assert small.retries > 0


@pytest.mark.gpu
def test_partition_device_rbac_matches_single_gpu_engine():
    from keto_amd import check, synth
    from keto_amd.partition import PartitionedEngine
    w = synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=20000, seed=9)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    want = check.Engine(snap).check_ids(roots, targets)
    for direction in ("forward", "backward"):
        np.testing.assert_array_equal(PartitionedEngine(snap, device=0, direction=direction).check_ids(roots, targets),
                                      want)
    eng = PartitionedEngine(snap, device=0, max_words_per_round=32)  # auto: trial rounds, then one direction
    got = eng.check_ids(roots, targets)
    np.testing.assert_array_equal(got, want)
    assert set(eng._trial) == {0, 1}
    orc = randgraph.oracle_store_columns(w.namespaces, w.columns)
    np.testing.assert_array_equal(got[:3000], orc.check_batch(w.requests(range(3000)), nthreads=8).astype(bool))


@pytest.mark.gpu
def test_partition_device_two_ranks_share_gpu():
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")
    namespaces, rows, reqs = _case(64)
    want = _want(namespaces, rows, reqs)
    got, rec = _run_ranks(2, 64, device_steps=True, port=29650)
    for g in got:
        np.testing.assert_array_equal(g, want)
    assert all(r[0] > 0 for r in rec)
