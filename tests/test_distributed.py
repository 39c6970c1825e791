"""Multi-rank (gloo, CPU) checks of the pool-sharded pass.

Two ranks each take the pools `assign_pools` gives them, insert only their
shard into a matchmaker (the CPU oracle here: the GPU path is the same C ABI),
run one interval pass, and gather the groups to rank 0, which checks that the
merged result is identical — groups, entry order and global group order — to a
single pass over the whole ticket set.  This is the property the multi-GPU
bench relies on.
"""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, config, n, q):
    import harness
    import sharding
    from nakama_amd import capi, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        npools = synth.N_POOLS[config]
        sizes = [0] * npools
        for i in range(n):
            sizes[synth.pool_of(config, i)] += 1
        mine = sharding.assign_pools(sizes, world)[rank]
        ts = synth.TicketSet(config, n, pool_mask=sharding.pool_mask(mine))
        mm = capi.Matchmaker(harness.oracle_lib(), max_intervals=2)
        ts.insert_into(mm)
        groups = mm.Process()
        created = {ts.ticket_id(k): ts.tickets[k].created_at for k in range(ts.n)}
        gathered = [None] * world
        dist.all_gather_object(gathered, (groups, created, mine, ts.n))
        if rank == 0:
            q.put(gathered)
        mm.close()
        ts.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("config,n", [(3, 900), (4, 1200)])
def test_pool_sharded_pass_equals_global_pass(config, n):
    import harness
    import sharding
    from nakama_amd import capi, synth
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, config, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # shards are disjoint and cover the set
    pools = [set(g[2]) for g in gathered]
    assert not (pools[0] & pools[1])
    assert sum(g[3] for g in gathered) == n
    created = {}
    for g in gathered:
        created.update(g[1])
    merged = sharding.merge_groups([g[0] for g in gathered], created)
    # single global pass
    ts = synth.TicketSet(config, n)
    mm = capi.Matchmaker(harness.oracle_lib(), max_intervals=2)
    try:
        ts.insert_into(mm)
        ref = mm.Process()
    finally:
        mm.close()
        ts.close()
    assert merged == ref


def test_assign_pools_balanced_and_deterministic():
    import sharding
    sizes = [125, 124, 130, 126, 119, 127, 125, 124]
    a = sharding.assign_pools(sizes, 4)
    assert sorted(p for b in a for p in b) == list(range(8))
    loads = [sum(sizes[p] for p in b) for b in a]
    assert max(loads) - min(loads) <= max(sizes)
    assert a == sharding.assign_pools(sizes, 4)


def _shard_worker(rank, world, port, config, n, q):
    """bench.py's multi-GPU workload: rank r owns shard instance r whole."""
    import harness
    from nakama_amd import capi, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ts = synth.TicketSet(config, n, first=rank * n, shard=rank)
        mm = capi.Matchmaker(harness.oracle_lib(), max_intervals=2)
        ts.insert_into(mm)
        groups = mm.Process()
        created = {ts.ticket_id(k): ts.tickets[k].created_at for k in range(ts.n)}
        matched = sum(len({t for t, _ in g}) for g in groups)
        tot = [None] * world
        dist.all_gather_object(tot, (groups, created, matched))
        if rank == 0:
            q.put(tot)
        mm.close()
        ts.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("config,n", [(3, 700), (4, 800)])
def test_shard_instances_equal_one_global_pass(config, n):
    """N ranks each running one disjoint instance of the config (bench.py's
    weak-scaling workload) produce exactly the groups of a single pass over
    all N instances together: the instances share no pool, so no group can
    span GPUs and no collective is needed in the data path."""
    import harness
    import sharding
    from nakama_amd import capi, synth
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, config, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    created = {}
    for g in gathered:
        created.update(g[1])
    merged = sharding.merge_groups([g[0] for g in gathered], created)
    mm = capi.Matchmaker(harness.oracle_lib(), max_intervals=2)
    sets = [synth.TicketSet(config, n, first=r * n, shard=r) for r in range(world)]
    try:
        for ts in sets:
            ts.insert_into(mm)
        ref = mm.Process()
    finally:
        mm.close()
        for ts in sets:
            ts.close()
    assert merged == ref
    assert sum(g[2] for g in gathered) == sum(len({t for t, _ in g}) for g in ref) > 0


def _merge_worker(rank, world, port, n_groups, reps, q):
    """ClusterMatchmaker.merge_keys over gloo on synthetic keys: rank r's
    groups at CreatedAt keys interleaved with every other rank's (C3's
    pools: every rank's groups spread over the whole time range)."""
    import time

    import numpy as np

    from nakama_amd import cluster
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["LOCAL_WORLD_SIZE"] = str(world)  # as torchrun sets it: the ranks split the host's cores
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(1000 + rank)
        # distinct keys across ranks (key % world == rank), ascending per rank
        keys = np.sort(rng.choice(np.arange(4 * n_groups, dtype=np.int64), n_groups, replace=False)) * world + rank
        cm = cluster.ClusterMatchmaker(None, dist, ("properties.mode", "properties.region"))
        times, comm, cmerge = [], [], []
        for _ in range(reps):
            cp = cluster.ClusterPass()
            dist.barrier()
            t0 = time.perf_counter()
            cm.merge_keys(cp, keys, 10 * n_groups, 17 * n_groups)
            times.append(1e3 * (time.perf_counter() - t0))
            comm.append(cp.local_stats["merge_comm_ms"])
            cmerge.append(cp.local_stats["merge_c_ms"])
        got = [None] * world
        dist.all_gather_object(got, (keys, cp.positions, cp.n_groups, times, comm, cmerge))
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_groups", [(8, 175_000), (2, 20_000)])
def test_cluster_merge_at_c3_volume(world, n_groups):
    """The pool-sharded merge (two all-gathers, mm_merge_positions_strided,
    one all-reduce) at world 8 with C3's group volume per rank (175k groups
    of a 1M-ticket pass): every group's global position is its key's rank in
    the merged key list.  Prints the merge time (rank 0's median, gloo on the
    host: DESIGN.md §7 records it)."""
    import numpy as np
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_merge_worker, args=(r, world, port, n_groups, 5, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    allk = np.concatenate([g[0] for g in got])
    allp = np.concatenate([g[1] for g in got])
    assert got[0][2] == world * n_groups
    assert np.array_equal(np.sort(allp), np.arange(world * n_groups))
    assert np.array_equal(allk[np.argsort(allp)], np.sort(allk))
    def med(x):
        return sorted(x)[len(x) // 2]
    print(f"\ncluster merge world {world} x {n_groups} groups: rank-0 median {med(got[0][3]):.2f} ms "
          f"(collectives {med(got[0][4]):.2f}, C merge {med(got[0][5]):.2f}; all ranks' C merge: "
          f"{[round(med(g[5]), 2) for g in got]})")
