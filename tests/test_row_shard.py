"""The row-sharded mode (include/nakama_cluster.h, cluster.RowShardedMatchmaker).

Workloads whose searches cross pools (config 9: C2's skill windows with no
region must; the mixed and RevPrecision workloads) cannot be split by pool.
Every rank then holds the whole ticket set, each batch's searches are cut
into one block per rank, and the blocks' results (result records, hit lists,
RevPrecision flags, pair matrices) are exchanged before the replicated
replay.  Every rank's groups and post-pass state must equal one oracle pass
over the whole set.  GPU tests: two ranks on the one-GPU box over the host
transport (gloo), and the RCCL transport at world 1 (RCCL cannot put two
ranks on one device; the driver's multi-GPU node runs it for real).
"""
import os
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_cluster import _free_port, _wait  # noqa: E402


def row_worker(rank, world, port, config, n, passes, cfg, transport, use_product, q, backend="gloo", env=None):
    os.environ.update(env or {})
    import harness
    from nakama_amd import capi, cluster, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":
        import torch
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if use_product:
            import nakama_amd
            lib = nakama_amd.load_library()
        else:
            lib = harness.oracle_lib()
        mm = capi.Matchmaker(lib, **cfg)
        rm = cluster.RowShardedMatchmaker(mm, dist, transport=transport)
        lo, hi = n * rank // world, n * (rank + 1) // world
        ts = synth.TicketSet(config, hi - lo, first=lo)
        rm.Insert(ts.ptr(), ts.n)
        out = []
        for _ in range(passes):
            r = rm.Process()
            out.append((r.groups, [(t.ticket, t.intervals) for t in rm.Extract()], mm.active_count(), r.eval_kernel))
        allout = [None] * world
        dist.all_gather_object(allout, (out, rm.gather_bytes))
        if rank == 0:
            q.put(allout)
        mm.close()
        ts.close()
    finally:
        dist.destroy_process_group()


def run_rows(config, n, passes, cfg, transport, use_product, world=2, backend="gloo", env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=row_worker,
                         args=(r, world, port, config, n, passes, cfg, transport, use_product, q, backend, env))
             for r in range(world)]
    for p in procs:
        p.start()
    res = _wait(q, procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def oracle_passes(config, n, passes, cfg):
    import harness
    from nakama_amd import capi, synth
    ts = synth.TicketSet(config, n)
    mm = capi.Matchmaker(harness.oracle_lib(), **cfg)
    try:
        ts.insert_into(mm)
        return [(mm.Process(), [(t.ticket, t.intervals) for t in mm.Extract()], mm.active_count())
                for _ in range(passes)]
    finally:
        mm.close()
        ts.close()


def test_replicas_equal_single_pass():
    """CPU: the replication plumbing (every rank inserts every rank's slice in
    rank order) over the oracle, no split: each replica equals one pass."""
    cfg = dict(max_intervals=2)
    allout = run_rows(9, 600, 2, cfg, None, False)
    want = oracle_passes(9, 600, 2, cfg)
    for out, _ in allout:
        assert [(g, s, a) for g, s, a, _ in out] == want


@pytest.mark.gpu
@pytest.mark.parametrize("config,n,passes,mi,rev", [(9, 3000, 2, 2, False), (6, 1000, 3, 3, False),
                                                     (5, 800, 2, 2, True), (7, 800, 2, 2, False)])
def test_row_sharded_host_transport(config, n, passes, mi, rev):
    cfg = dict(max_intervals=mi, rev_precision=rev)
    allout = run_rows(config, n, passes, cfg, "host", True)
    want = oracle_passes(config, n, passes, cfg)
    for out, nbytes in allout:
        assert [(g, s, a) for g, s, a, _ in out] == want
        assert nbytes > 0  # the blocks really were exchanged


@pytest.mark.gpu
@pytest.mark.parametrize("config,n", [(4, 12_000), (3, 9_000)])
def test_row_sharded_hashed_scan_host_transport(config, n):
    """C4's shape (64 mode x region pools, its BASELINE mode: row-sharded)
    and C3's: every batch's pool signatures run as one hashed scan split by
    candidate chunks — each rank scans its block, the chunk outputs and
    counts are all-gathered, every rank places every list — equal to one
    oracle pass, with eval_kernel 4 (mscan_hash_kernel) on every rank."""
    cfg = dict(max_intervals=2)
    allout = run_rows(config, n, 2, cfg, "host", True, env={"NKM_KERNEL": "mscan"})
    want = oracle_passes(config, n, 2, cfg)
    for out, nbytes in allout:
        assert [(g, s, a) for g, s, a, _ in out] == want
        assert out[0][3] == 4
        assert nbytes > 0


@pytest.mark.gpu
def test_row_sharded_rccl_transport_world1():
    """The RCCL path (grouped in-place ncclBroadcast on the library's stream)
    at world 1 — the exchange runs, trivially — equal to the oracle."""
    cfg = dict(max_intervals=2)
    allout = run_rows(9, 2000, 2, cfg, "rccl", True, world=1)
    want = oracle_passes(9, 2000, 2, cfg)
    out, _ = allout[0]
    assert [(g, s, a) for g, s, a, _ in out] == want
