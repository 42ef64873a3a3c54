"""Two-tier partitioned mode (include/ketogpu.h "two-tier", keto_amd/csrc/tier.cpp): the
core gathered on every rank, the queries / replies protocol and the evaluation, against
the oracle.

CPU tests load real shards (the C++ loader) with world_size 1, 2 and 3 over gloo and run
the NATIVE protocol with each rank's device steps played by tests/tier_cpu.py; every rank
passes its own slice of the requests.  The GPU tests run the HIP steps (the lite unit over
the local core, device_engine.hip tier_* kernels) at world 1 (rows read in place), over a
real RCCL communicator of one rank (the exchange path through ncclSend/ncclRecv), and
with two ranks sharing the box's GPU over gloo."""
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from keto_amd import _lib as L
from keto_amd import persistence
from tests.test_partition import _batches, _case, _load, _want


def _slices(n, world):
    """rank k's requests: a strided slice, with unequal sizes"""
    return [np.arange(k, n, world) for k in range(world)]


def _tier_worker(rank, world, port, seed, out_dir, device_steps, max_batch, force_overflow=False):
    import torch.distributed as dist
    if force_overflow:
        os.environ["KETOGPU_TEST_TIER_OVERFLOW"] = "1"
    from keto_amd.partition import Core, TieredEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        namespaces, rows, reqs = _case(seed)
        sh = _load(namespaces, rows)
        roots, targets, status = sh.resolve_batch(persistence.request_columns(reqs))
        idx = _slices(len(reqs), world)[rank]
        if rank == world - 1 and world > 2:
            idx = idx[:0]  # one rank with no requests still joins every collective
        if device_steps:
            eng = TieredEngine(sh, device=0, comm=sh.native_comm(0, host_steps=True), max_batch=max_batch)
        else:
            from tests.tier_cpu import CpuTier
            core = Core(sh, sh.native_comm(host_steps=True))
            eng = TieredEngine(sh, local=CpuTier(sh.view(), core.view()), core=core, max_batch=max_batch)
            cv = core.view()
            np.save(os.path.join(out_dir, f"core{rank}.npy"),
                    np.concatenate([[cv["num_interior"], len(cv["f_col"]), len(cv["b_col"])]] +
                                   [cv[k].astype(np.int64) for k in ("f_off", "f_col", "b_off", "b_col")]))
        got = eng.check_ids(roots[idx], targets[idx])
        st = eng.stats()
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), np.stack([idx, got.astype(np.int64)]))
        np.save(os.path.join(out_dir, f"stats{rank}.npy"),
                np.array([st["queries_sent"], st["records_sent"], st["records_received"], st["batches"],
                          st["overflow_requests"], st["fallback_calls"]]))
        eng.close()
    finally:
        dist.destroy_process_group()


def _run_tier(world, seed, port, device_steps=False, max_batch=0, force_overflow=False):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_tier_worker, args=(world, port, seed, d, device_steps, max_batch, force_overflow),
                           nprocs=world, join=True, start_method="spawn")
        got = [np.load(os.path.join(d, f"rank{r}.npy")) for r in range(world)]
        stats = [np.load(os.path.join(d, f"stats{r}.npy")) for r in range(world)]
        cores = [np.load(os.path.join(d, f"core{r}.npy")) for r in range(world)] if not device_steps else []
    return got, stats, cores


def test_core_single_rank_is_the_interior_rows():
    """world 1: the core is exactly the shard's interior rows (forward and backward)"""
    from keto_amd.partition import Core
    namespaces, rows, _ = _case(80)
    sh = _load(namespaces, rows)
    v, c = sh.view(), Core(sh).view()
    nil = v["owned_interior"]
    assert c["num_interior"] == v["num_interior"] == nil
    np.testing.assert_array_equal(c["f_off"], v["lf_off"][:nil + 1])
    np.testing.assert_array_equal(c["f_col"], v["lf_col"][:int(v["lf_off"][nil])])
    np.testing.assert_array_equal(c["b_off"], v["lb_off"])
    np.testing.assert_array_equal(c["b_col"], v["lb_col"])
    assert c["bytes"] == 16 * (len(c["f_col"]) + len(c["b_col"]))
    with pytest.raises(L.KetoError) as e:  # a budget below the core's records
        Core(sh, budget=max(c["bytes"] - 1, 1))
    assert e.value.code == L.ENOMEM


def test_tier_protocol_single_rank_cpu():
    from keto_amd.partition import Core, TieredEngine
    from tests.tier_cpu import CpuTier
    namespaces, rows, reqs = _case(81)
    sh = _load(namespaces, rows)
    core = Core(sh)
    eng = TieredEngine(sh, local=CpuTier(sh.view(), core.view()), core=core, max_batch=128)
    roots, targets, _ = sh.resolve_batch(persistence.request_columns(reqs))
    want = _want(namespaces, rows, reqs)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    st = eng.stats()
    assert st["batches"] == (len(reqs) + 127) // 128 and st["queries_sent"] == 0  # world 1: no exchange
    assert want.any() and not want.all()


@pytest.mark.parametrize("world,seed,max_batch", [(2, 82, 0), (3, 83, 64)])
def test_tier_protocol_multi_rank_gloo(world, seed, max_batch):
    """each rank checks its own requests (one rank of three has none; 64-request steps:
    ranks with fewer steps run empty ones); the core is identical on every rank"""
    namespaces, rows, reqs = _case(seed)
    want = _want(namespaces, rows, reqs)
    got, stats, cores = _run_tier(world, seed, 29700 + 10 * world, max_batch=max_batch)
    seen = 0
    for g in got:
        idx, ans = g
        np.testing.assert_array_equal(ans.astype(bool), want[idx])
        seen += len(idx)
    assert seen == len(reqs) - (len(_slices(len(reqs), world)[-1]) if world > 2 else 0)
    assert all(s[0] > 0 for s in stats[:2]) and sum(s[1] for s in stats) == sum(s[2] for s in stats) > 0
    assert len({s[3] for s in stats}) == 1  # every rank ran the same number of steps
    for c in cores[1:]:
        np.testing.assert_array_equal(c, cores[0])
    # the same rows as one rank's core (ids differ: the layout interleaves the ranks)
    from keto_amd.partition import Core
    single = Core(_load(namespaces, rows)).view()
    assert (cores[0][1], cores[0][2]) == (len(single["f_col"]), len(single["b_col"]))
    assert cores[0][0] >= single["num_interior"]


def _fail_tier_worker(rank, world, port, out_dir):
    """rank 1 sends an id outside the layout: every rank raises (no rank is left waiting
    in a collective), rank 1 with EINVAL, and the next batch is answered normally"""
    import torch.distributed as dist
    from keto_amd.partition import Core, TieredEngine
    from tests.tier_cpu import CpuTier
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        namespaces, rows, reqs = _case(84)
        sh = _load(namespaces, rows)
        roots, targets, _ = sh.resolve_batch(persistence.request_columns(reqs))
        core = Core(sh, sh.native_comm(host_steps=True))
        eng = TieredEngine(sh, local=CpuTier(sh.view(), core.view()), core=core)
        idx = _slices(len(reqs), world)[rank]
        r, t = roots[idx].copy(), targets[idx].copy()
        if rank == 1:
            r[3] = 1 << 30
        codes = []
        try:
            eng.check_ids(r, t)
            codes.append(0)
        except L.KetoError as e:
            codes.append(e.code)
        codes.append(int(eng.check_ids(roots[idx], targets[idx]).sum()))
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), np.array(codes))
    finally:
        dist.destroy_process_group()


def test_tier_invalid_id_on_one_rank_fails_every_rank():
    namespaces, rows, reqs = _case(84)
    want = _want(namespaces, rows, reqs)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_fail_tier_worker, args=(2, 29760, d), nprocs=2, join=True, start_method="spawn")
        codes = [np.load(os.path.join(d, f"rank{r}.npy")) for r in range(2)]
    assert codes[1][0] == L.EINVAL and codes[0][0] != 0
    for k in range(2):
        assert codes[k][1] == int(want[_slices(len(reqs), 2)[k]].sum())


def _c5_tier_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from keto_amd import synth
    from keto_amd.partition import Core, Shard, TieredEngine
    from tests.tier_cpu import CpuTier
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = synth.config5(users=30000, groups=3000, docs=6000, tuples=150000, checks=1500, seed=17)
        sh = Shard.load(w.namespaces, lambda: w.batches(4093))
        roots, targets, st = sh.resolve_batch(w.request_batch())
        core = Core(sh)
        cv = core.view()
        eng = TieredEngine(sh, local=CpuTier(sh.view(), cv), core=core)
        idx = _slices(len(roots), world)[rank]
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), np.stack([idx, eng.check_ids(roots[idx], targets[idx])]))
        np.save(os.path.join(out_dir, f"core{rank}.npy"),
                np.array([cv["num_interior"], len(cv["f_col"]), len(cv["b_col"]), sh.stats()["rows"]]))
    finally:
        dist.destroy_process_group()


def test_tier_config5_stream_two_ranks_match_oracle():
    """config #5's stream read by two ranks; the core is group nesting only (a small share
    of the rows); each rank's own requests against the oracle over the same stream"""
    from keto_amd import synth
    from oracle import oracle as O
    w = synth.config5(users=30000, groups=3000, docs=6000, tuples=150000, checks=1500, seed=17)
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(4093):
        st.add_columnar(cols)
    want = st.finalize(presorted=True).check_batch(w.requests(range(w.n_checks)), nthreads=4).astype(bool)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_c5_tier_worker, args=(2, 29770, d), nprocs=2, join=True, start_method="spawn")
        got = [np.load(os.path.join(d, f"rank{r}.npy")) for r in range(2)]
        cores = [np.load(os.path.join(d, f"core{r}.npy")) for r in range(2)]
    for idx, ans in got:
        np.testing.assert_array_equal(ans.astype(bool), want[idx])
    np.testing.assert_array_equal(cores[0], cores[1])
    assert cores[0][1] + cores[0][2] < 0.1 * cores[0][3]  # the core is a small part of the rows
    assert want[w.chk_pos.astype(bool)].all() and not want.all()


# --------------------------------------------------------------------- GPU
def _need_gpu():
    if L.lib().ketogpu_device_count() < 1:
        pytest.fail("no HIP device visible")


# plan label (the default: owners reply with label lists, one intersection per request)
# and the row exchange + LDS units (KETOGPU_TIER_LABEL=0)
LABEL = pytest.mark.parametrize("label", ["1", "0"], ids=["label", "rows"])


def _mode(monkeypatch, label):
    monkeypatch.setenv("KETOGPU_TIER_LABEL", label)


def _check_mode(st, label):
    assert st["label"] == int(label)
    if label == "1":
        assert st["label_words"] > 0 and st["overflow_requests"] == 0


@pytest.mark.gpu
@LABEL
@pytest.mark.parametrize("seed", [91, 92])
def test_tier_device_single_rank(seed, label, monkeypatch):
    """world 1: rows (or label lists) read in place; random networks with poisoned pages,
    several steps, pinned and pageable requests"""
    from keto_amd import check
    from keto_amd.partition import TieredEngine
    _need_gpu()
    _mode(monkeypatch, label)
    namespaces, rows, reqs = _case(seed, n_rows=1500, n_req=3000)
    sh = _load(namespaces, rows)
    want = _want(namespaces, rows, reqs)
    roots, targets, _ = sh.resolve_batch(persistence.request_columns(reqs))
    eng = TieredEngine(sh, device=0, max_batch=1024)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    pr, pt = check.pinned(roots), check.pinned(targets)
    np.testing.assert_array_equal(eng.check_ids(pr.array, pt.array), want)
    st = eng.stats()
    assert st["batches"] == 2 * 3 and st["rows_opened"] > 0 and st["overflow_requests"] == 0
    _check_mode(st, label)
    # an id outside the layout fails the call; the engine answers the next batch
    r = roots.copy()
    r[5] = 1 << 30
    with pytest.raises(L.KetoError) as e:
        eng.check_ids(r, targets)
    assert e.value.code == L.EINVAL
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)


@pytest.mark.gpu
@LABEL
def test_tier_device_config5_matches_oracle(label, monkeypatch):
    """config #5's shape through the partition-aware loader, the core and the HIP steps,
    every request against the oracle (and the per-level engine agrees)"""
    from keto_amd import synth
    from keto_amd.partition import PartitionedEngine, Shard, TieredEngine
    _need_gpu()
    _mode(monkeypatch, label)
    w = synth.config5(users=100000, groups=10000, docs=40000, tuples=1_000_000, checks=20000, seed=23)
    from oracle import oracle as O
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(1 << 16):
        st.add_columnar(cols)
    want = st.finalize(presorted=True).check_batch(w.requests(range(w.n_checks)), nthreads=8).astype(bool)
    sh = Shard.load(w.namespaces, lambda: w.batches(1 << 16))
    roots, targets, status = sh.resolve_batch(w.request_batch())
    eng = TieredEngine(sh, device=0)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    _check_mode(eng.stats(), label)
    np.testing.assert_array_equal(PartitionedEngine(sh, device=0, direction="backward").check_ids(roots, targets),
                                  want)
    assert want[w.chk_pos.astype(bool)].all()


@pytest.mark.gpu
@LABEL
def test_tier_device_power_law_cascade(label, monkeypatch):
    """power-law nesting (config #4's shape, small): large closures take the larger-table
    stages and, past them, the per-level engine (rows mode), or long label lists read past
    their LDS copies (label mode); every answer against the oracle"""
    from keto_amd import synth
    from keto_amd.partition import Shard, TieredEngine
    _need_gpu()
    _mode(monkeypatch, label)
    w = synth.social(users=20000, groups=4000, tuples=200_000, checks=20000, seed=31)
    want = randgraph_want(w)
    sh = Shard.load(w.namespaces, lambda: iter([w.columns]))
    roots, targets, status = sh.resolve_batch(w.request_batch())
    eng = TieredEngine(sh, device=0)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    _check_mode(eng.stats(), label)


def randgraph_want(w):
    from tests import randgraph
    return randgraph.oracle_store_columns(w.namespaces, w.columns).check_batch(
        w.requests(range(w.n_checks)), nthreads=8).astype(bool)


@pytest.mark.gpu
@LABEL
@pytest.mark.parametrize("loop_self,one_wait", [(False, "1"), (False, "0"), (True, "1")],
                         ids=["copy-one-wait", "copy-general", "rccl-self"])
def test_tier_device_rccl_world1_matches_oracle(loop_self, one_wait, label, monkeypatch):
    """a real RCCL communicator of one rank: the exchange path (queries, replies, seed
    records from the received rows) against the oracle.  By default the own segment of each
    all-to-all is a copy-engine DMA and the world-1 count gathers are skipped, so only the
    loader's ncclAllGather runs over RCCL; with KETOGPU_TEST_RCCL_SELF=1 every exchange is a
    grouped ncclSend/ncclRecv to the rank itself and every count gather an ncclAllGather —
    the data path of a multi-GPU run, executed on one GPU (counted by the communicator).
    Plan label at world 1 without loop_self runs the one-wait step (TierDevice::step_world1:
    pair slots, no counts; its first step outgrows the reply buffer and is evaluated again)
    unless KETOGPU_TIER_ONE_WAIT=0 (the general protocol, buffers swapped)"""
    monkeypatch.setenv("KETOGPU_TIER_ONE_WAIT", one_wait)
    if loop_self:
        monkeypatch.setenv("KETOGPU_TEST_RCCL_SELF", "1")
    _mode(monkeypatch, label)
    from keto_amd import synth
    from keto_amd.partition import NativeComm, Shard, TieredEngine
    _need_gpu()
    w = synth.config5(users=50000, groups=5000, docs=20000, tuples=400_000, checks=12000, seed=29)
    from oracle import oracle as O
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(1 << 16):
        st.add_columnar(cols)
    want = st.finalize(presorted=True).check_batch(w.requests(range(w.n_checks)), nthreads=8).astype(bool)
    comm = NativeComm(device=0, kind="rccl")
    sh = Shard.load(w.namespaces, lambda: w.batches(1 << 16), native_comm=comm)
    roots, targets, status = sh.resolve_batch(w.request_batch(), comm)
    eng = TieredEngine(sh, device=0, comm=comm, max_batch=4096)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    # answers into pinned words (written in place by the emit launch at world 1)
    from keto_amd import check
    pb = check.PinnedBuffer((len(roots) + 63) // 64, np.uint64)
    eng.check_ids_raw(np.ascontiguousarray(roots, np.uint32), np.ascontiguousarray(targets, np.uint32), pb.array)
    np.testing.assert_array_equal(check.unpack_bits(pb.array.copy(), len(roots)), want)
    s = eng.stats()
    assert s["queries_sent"] > 0 and s["records_sent"] == s["records_received"] > 0
    _check_mode(s, label)
    cs = comm.stats()
    assert cs["rccl"] == 1 and cs["loop_self"] == int(loop_self) and cs["allgathers"] > 0
    if loop_self:  # two all-to-alls (queries, replies) and their count gathers per step
        steps = (len(roots) + 4095) // 4096
        assert cs["sends"] >= 2 * steps and cs["recvs"] == cs["sends"] and cs["allgathers"] >= 2 * steps
        unit = 4 if label == "1" else 8  # label replies are 4-byte words, row replies 8-byte records
        assert cs["bytes_sent"] >= 8 * s["queries_sent"] + unit * s["records_sent"]
    else:
        assert cs["sends"] == 0 and cs["recvs"] == 0


@pytest.mark.gpu
@LABEL
@pytest.mark.parametrize("world", [2, 3])
def test_tier_device_two_ranks_share_gpu(label, world, monkeypatch):
    """two (three) ranks on the box's GPU over gloo: device steps, host transport (staged);
    with three ranks every label reply segment layout has a middle segment (the row protocol
    at world 3 is covered by the CPU steps' gloo tests)"""
    if world == 3 and label == "0":
        pytest.skip("row protocol at world 3: CPU steps (test_tier_protocol_multi_rank_gloo)")
    _need_gpu()
    _mode(monkeypatch, label)
    namespaces, rows, reqs = _case(85)
    want = _want(namespaces, rows, reqs)
    got, stats, _ = _run_tier(world, 85, 29790 + world, device_steps=True)
    for idx, ans in got:
        np.testing.assert_array_equal(ans.astype(bool), want[idx])
    # every rank with requests sent queries; at world 3 the last rank has none (_tier_worker)
    # and still answers the others' queries as an owner
    assert all(s[0] > 0 for s in (stats if world == 2 else stats[:-1]))
    assert world == 2 or (stats[-1][0] == 0 and stats[-1][1] > 0)


@pytest.mark.gpu
def test_tier_device_fallback_to_per_level_engine(monkeypatch):
    """KETOGPU_TEST_TIER_OVERFLOW=1: every request reported unfinished by the LDS stages, so
    the per-level engine (built on first need from the same shard) answers all of them —
    one rank, then two ranks sharing the GPU over gloo (the overflow lists gathered from
    both ranks, each rank keeping its own answers)"""
    from keto_amd.partition import TieredEngine
    _need_gpu()
    namespaces, rows, reqs = _case(86, n_rows=1200, n_req=1500)
    want = _want(namespaces, rows, reqs)
    sh = _load(namespaces, rows)
    roots, targets, _ = sh.resolve_batch(persistence.request_columns(reqs))
    monkeypatch.setenv("KETOGPU_TEST_TIER_OVERFLOW", "1")
    eng = TieredEngine(sh, device=0)
    np.testing.assert_array_equal(eng.check_ids(roots, targets), want)
    st = eng.stats()
    assert st["fallback_calls"] == 1 and st["overflow_requests"] == len(reqs)
    monkeypatch.delenv("KETOGPU_TEST_TIER_OVERFLOW")
    got, stats, _ = _run_tier(2, 86, 29795, device_steps=True, force_overflow=True)
    for idx, ans in got:
        np.testing.assert_array_equal(ans.astype(bool), _case_want(86, idx))  # the workers' _case(86)
    assert all(s[5] >= 1 and s[4] > 0 for s in stats)


def _case_want(seed, idx):
    namespaces, rows, reqs = _case(seed)
    return _want(namespaces, rows, reqs)[idx]
