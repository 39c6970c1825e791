"""One `server.Matchmaker` over the GPUs of a node: the pool-sharded front.

The reference runs a single LocalMatchmaker per node; every Add/Insert/
Remove* reaches it and one Process() pass covers every ticket
(server/matchmaker.go:169-183, constructed at main.go:160).  Here one process
per GPU holds a rank-local handle (libnakama_mm, `mm_config.device`) and
`ClusterMatchmaker` keeps the single-instance contract over all of them.

Routing (include/nakama_cluster.h).  A ticket belongs to the pool named by
the keyword values its query requires on the configured pool fields, which
must also be its own property values (`mm_route_keys`).  Searches of a pool
only hit that pool's documents and only that pool's searches hit them, so the
reference's pass over all tickets is the interleaving of independent per-pool
passes (matchmaker_process.go:38-330: selection, Intervals and hit lists
never cross a pool).  Whole pools are placed on ranks by a directory that
every rank updates identically (online longest-processing-time: a new pool
goes to the least-loaded rank), and tickets move to their owner with one
all-to-all of packed records (RCCL over xGMI when the group is "nccl").

Process.  Every rank runs its own pass — no data-path collective — and the
reference's group order is recovered by merging the ranks' group lists on
the searching ticket's (CreatedAt, Ticket) (`mm_merge_positions`; the keys
come back in `mm_matched.group_created`): one all-gather of 8 B per group,
after which every rank knows the global position of each of its groups
(`ClusterPass.positions`, a linear merge on each rank).  A group's tickets all
live on one rank, which owns its delivery; `gather_groups()` materialises the
merged list on rank 0 for callers that need it whole (tests).

Every method is a collective: all ranks call it, in the same order.  Tickets
that are not partitionable on the pool fields (a query that does not pin a
pool field to the ticket's own value) are returned to the caller by Insert
and not inserted — a deployment with cross-pool queries uses the
row-sharded mode instead.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT_SO = os.path.join(ROOT, "nakama_amd", "libnakama_mm.so")

_router = None


def router_lib(path: str = PRODUCT_SO) -> C.CDLL:
    """The routing entry points of include/nakama_cluster.h (host-only: they
    load and run without a GPU)."""
    global _router
    if _router is None:
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = C.CDLL(path, mode=C.RTLD_LOCAL)
        lib.mm_route_keys.restype = C.c_int32
        lib.mm_route_keys.argtypes = [C.POINTER(capi.mm_ticket), C.c_int32, C.POINTER(C.c_char_p), C.c_int32,
                                      C.POINTER(C.c_uint64)]
        lib.mm_pack_tickets.restype = C.c_int64
        lib.mm_pack_tickets.argtypes = [C.POINTER(capi.mm_ticket), C.POINTER(C.c_int32), C.c_int32, C.c_void_p,
                                        C.c_int64]
        lib.mm_unpack_tickets.restype = C.c_void_p
        lib.mm_unpack_tickets.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_int32),
                                          C.POINTER(C.POINTER(capi.mm_ticket))]
        lib.mm_free_unpacked.argtypes = [C.c_void_p]
        lib.mm_merge_positions.restype = C.c_int32
        lib.mm_merge_positions.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        lib.mm_count_tickets.restype = C.c_int64
        lib.mm_count_tickets.argtypes = [C.c_void_p]
        lib.mm_merge_positions_strided.restype = C.c_int32
        lib.mm_merge_positions_strided.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_int32,
                                                   C.c_void_p]
        lib.mm_merge_positions_ex.restype = C.c_int32
        lib.mm_merge_positions_ex.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                              C.c_void_p]
        _router = lib
    return _router


CLUSTER_SYMBOLS = ("mm_route_keys", "mm_pack_tickets", "mm_unpack_tickets", "mm_free_unpacked",
                   "mm_merge_positions", "mm_merge_positions_strided", "mm_merge_positions_ex", "mm_count_tickets", "mm_shard_rows", "mm_rccl_unique_id", "mm_shard_rows_rccl",
                   "mm_create_multi", "mm_multi_info", "mm_device_numa_node")


def route_keys(tickets, n: int, pool_fields: Sequence[str]) -> np.ndarray:
    """uint64 pool key per ticket (0: not partitionable on pool_fields)."""
    L = router_lib()
    keys = np.zeros(max(n, 1), dtype=np.uint64)
    fs = (C.c_char_p * len(pool_fields))(*[f.encode() for f in pool_fields])
    if n:
        L.mm_route_keys(tickets, n, fs, len(pool_fields), keys.ctypes.data_as(C.POINTER(C.c_uint64)))
    return keys[:n]


def pack(tickets, idx: np.ndarray) -> np.ndarray:
    L = router_lib()
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    ip = idx.ctypes.data_as(C.POINTER(C.c_int32))
    need = L.mm_pack_tickets(tickets, ip, len(idx), None, 0)
    buf = np.empty(need, dtype=np.uint8)
    got = L.mm_pack_tickets(tickets, ip, len(idx), buf.ctypes.data, need)
    assert got == need
    return buf


class Unpacked:
    """Tickets decoded from packed records (owned by the library until close)."""

    def __init__(self, buf: np.ndarray):
        L = router_lib()
        self.n = C.c_int32(0)
        self.tickets = C.POINTER(capi.mm_ticket)()
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        self.h = L.mm_unpack_tickets(buf.ctypes.data if len(buf) else None, len(buf), C.byref(self.n),
                                     C.byref(self.tickets))
        if not self.h:
            raise ValueError("malformed ticket records")

    def close(self):
        if self.h:
            router_lib().mm_free_unpacked(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class ClusterPass:
    """One cluster-wide Process(): every rank's local result plus the global
    group order (rank 0)."""
    n_groups: int = 0              # all ranks
    matched_tickets: int = 0       # all ranks
    matched_presences: int = 0     # all ranks
    local: Optional[capi.ProcessResult] = None   # this rank's groups (when kept)
    positions: Optional[np.ndarray] = None       # global position of each of this rank's groups
    local_stats: Dict[str, float] = field(default_factory=dict)


class ClusterMatchmaker:
    """server.Matchmaker across the ranks of a torch.distributed group.

    local: this rank's handle (capi.Matchmaker over libnakama_mm on this
    rank's GPU, or any library with the same ABI); dist: torch.distributed
    (initialised); pool_fields: the query fields a pool is keyed on, e.g.
    ("properties.mode", "properties.region")."""

    def __init__(self, local: capi.Matchmaker, dist, pool_fields: Sequence[str], *, comm_device=None,
                 override_commit=None):
        """override_commit(local, candidates) -> committed result: with a
        MatchmakerOverride registered, the rank's hand-off of its processCustom
        candidates (frees them; returns mm_process_commit's library-owned
        result); default: local.override over the candidates as Python
        groups, then mm_process_commit.  The override runs per rank on that
        rank's candidates — exact for overrides that decide each pool on its
        own (a candidate group never spans pools), such as first-disjoint."""
        self.override_commit = override_commit
        self.local = local
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.pool_fields = list(pool_fields)
        self.comm_device = comm_device  # torch.device for "nccl" tensors, None for host (gloo)
        self.directory: Dict[int, int] = {}
        self.load = [0] * self.world
        self.owner_of: Dict[str, int] = {}  # rank 0, global override scope: ticket -> rank
        self._bufs: Dict[str, tuple] = {}  # merge staging buffers (host, device), reused across passes

    # ---- collectives over tensors ----
    def _t(self, arr: np.ndarray):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr))
        return t.to(self.comm_device) if self.comm_device is not None else t

    def _host(self, t) -> np.ndarray:
        return t.cpu().numpy() if self.comm_device is not None else t.numpy()

    def _all_gather_var(self, arr: np.ndarray) -> Tuple[np.ndarray, List[int]]:
        """Concatenation of every rank's 1-D array (ranks in order), and the counts."""
        import torch
        n = np.array([len(arr)], dtype=np.int64)
        sizes = [self._t(np.zeros(1, dtype=np.int64)) for _ in range(self.world)]
        self.dist.all_gather(sizes, self._t(n))
        counts = [int(self._host(s)[0]) for s in sizes]
        m = max(counts) if counts else 0
        pad = np.zeros(max(m, 1), dtype=arr.dtype)
        pad[:len(arr)] = arr
        outs = [self._t(np.zeros(max(m, 1), dtype=arr.dtype)) for _ in range(self.world)]
        self.dist.all_gather(outs, self._t(pad))
        parts = [self._host(o)[:c] for o, c in zip(outs, counts)]
        return (np.concatenate(parts) if parts else np.zeros(0, dtype=arr.dtype)), counts

    def _all_to_all_bytes(self, send: np.ndarray, splits: List[int]) -> np.ndarray:
        import torch
        sizes_in = self._t(np.array(splits, dtype=np.int64))
        sizes_out = self._t(np.zeros(self.world, dtype=np.int64))
        self.dist.all_to_all_single(sizes_out, sizes_in)
        out_splits = [int(x) for x in self._host(sizes_out)]
        recv = self._t(np.zeros(max(sum(out_splits), 1), dtype=np.uint8))
        self.dist.all_to_all_single(recv[:sum(out_splits)] if sum(out_splits) else recv[:0],
                                    self._t(send) if len(send) else self._t(np.zeros(0, dtype=np.uint8)),
                                    output_split_sizes=out_splits, input_split_sizes=splits)
        return self._host(recv)[:sum(out_splits)]

    # ---- routing ----
    def _place_new_pools(self, keys: np.ndarray):
        """Directory update, identical on every rank: the pools no rank had
        seen, largest first, each to the least-loaded rank."""
        ks = keys[keys != 0]
        uniq, cnt = np.unique(ks, return_counts=True)
        new = np.array([int(k) not in self.directory for k in uniq], dtype=bool) if len(uniq) else np.zeros(0, bool)
        gathered = [None] * self.world
        self.dist.all_gather_object(gathered, (uniq[new].tolist(), cnt[new].tolist()))
        tot: Dict[int, int] = {}
        for ks_r, cs_r in gathered:
            for k, c in zip(ks_r, cs_r):
                tot[int(k)] = tot.get(int(k), 0) + int(c)
        for k in sorted(tot, key=lambda k: (-tot[k], k)):
            r = min(range(self.world), key=lambda q: (self.load[q], q))
            self.directory[k] = r
            self.load[r] += tot[k]

    def owners(self, keys: np.ndarray) -> np.ndarray:
        """Owning rank of each pool key (-1: not partitionable / unknown)."""
        own = np.full(len(keys), -1, dtype=np.int32)
        if not self.directory or not len(keys):
            return own
        dk = np.fromiter(self.directory.keys(), dtype=np.uint64, count=len(self.directory))
        dr = np.fromiter(self.directory.values(), dtype=np.int32, count=len(self.directory))
        o = np.argsort(dk)
        dk, dr = dk[o], dr[o]
        pos = np.clip(np.searchsorted(dk, keys), 0, len(dk) - 1)
        hit = (dk[pos] == keys) & (keys != 0)
        own[hit] = dr[pos[hit]]
        return own

    def Insert(self, tickets, n: int) -> np.ndarray:
        """Insert (matchmaker.go:567-682) of this rank's ingest batch (an
        mm_ticket array): each ticket goes to its pool's rank.  Returns the
        indexes of the tickets that are not partitionable (not inserted)."""
        keys = route_keys(tickets, n, self.pool_fields)
        self._place_new_pools(keys)
        own = self.owners(keys)
        order = np.argsort(own, kind="stable")
        bounds = np.searchsorted(own[order], np.arange(self.world + 1), side="left")  # the -1s sort first
        parts, splits = [], []
        for r in range(self.world):
            idx = order[bounds[r]:bounds[r + 1]]
            buf = pack(tickets, idx) if len(idx) else np.zeros(0, dtype=np.uint8)
            parts.append(buf)
            splits.append(len(buf))
        send = np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)
        recv = self._all_to_all_bytes(send, splits)
        u = Unpacked(recv)
        try:
            if u.n.value:
                self.local._check(self.local.lib.mm_insert(self.local.h, u.tickets, u.n.value))
        finally:
            u.close()
        return np.nonzero(own < 0)[0]

    # ---- the pass ----
    def Process(self, keep_groups: bool = False) -> ClusterPass:
        """One interval pass on every rank, and the global position of every
        group in the reference's order.  keep_groups: also convert this rank's
        groups to Python (tests, delivery)."""
        import time
        t0 = time.perf_counter()
        out = self.local.process_call()
        err = None
        if out.is_candidates:  # processCustom: this rank's override hand-off
            out, err = self._override(out)
        if self.local.override is not None or self.override_commit is not None:
            # an override that raised on any rank fails the pass on every rank
            # (every rank takes part, with or without candidates of its own)
            flag = self._t(np.array([1 if err is not None else 0], dtype=np.int32))
            self.dist.all_reduce(flag, op=self.dist.ReduceOp.MAX)
            if int(self._host(flag)[0]):
                self.local.lib.mm_free_matched(self.local.h, C.byref(out))
                raise err if err is not None else RuntimeError("MatchmakerOverride failed on another rank")
        t1 = time.perf_counter()
        try:
            ng = out.n_groups
            keys = np.ctypeslib.as_array(out.group_created, (ng,)).copy() if ng else np.zeros(0, dtype=np.int64)
            res = None
            if keep_groups:
                res = capi.ProcessResult(capi.Matchmaker._groups(out), bool(out.is_candidates), out.n_expired,
                                         out.pass_ms, out.eval_ms, out.pair_evals, out.eval_bytes, out.eval_launches,
                                         out.n_batches, out.eval_kernel, out.full_lists, out.pairs_decided)
            _, tickets, pres, stats = self.local.summary_counts(out)
            t2 = time.perf_counter()
            cp = ClusterPass(local=res)

            def tie_ids():
                offs = out.group_offsets
                return [out.entries[offs[g + 1] - 1].ticket.decode() for g in range(ng)]
            self.merge_keys(cp, keys, tickets, pres, tie_ids)
        finally:
            self.local.lib.mm_free_matched(self.local.h, C.byref(out))
        t3 = time.perf_counter()
        cp.local_stats = {**cp.local_stats, "pass_ms": stats.pass_ms, "eval_ms": stats.eval_ms, "eval_bytes": stats.eval_bytes,
                          "pair_evals": stats.pair_evals, "pairs_decided": stats.pairs_decided,
                          "eval_launches": stats.eval_launches, "n_batches": stats.n_batches,
                          "eval_kernel": stats.eval_kernel, "local_call_ms": 1e3 * (t1 - t0),
                          "summary_ms": 1e3 * (t2 - t1), "merge_ms": 1e3 * (t3 - t2)}
        return cp

    def _staging(self, name: str, n: int, dtype):
        """A reusable host buffer of at least n elements (pinned when the
        collectives run on the device: the keys' copies then run at full PCIe
        rate and need no per-pass allocation) and its device twin."""
        import torch
        buf = self._bufs.get(name)
        if buf is None or buf[0].numel() < n:
            cap = max(n, 1024)
            host = torch.empty(cap, dtype=dtype, pin_memory=self.comm_device is not None)
            dev = torch.empty(cap, dtype=dtype, device=self.comm_device) if self.comm_device is not None else host
            buf = self._bufs[name] = (host, dev)
        return buf

    def merge_keys(self, cp: ClusterPass, keys: np.ndarray, tickets: int, pres: int, tie_ids=None):
        """The merge of a cluster pass: this rank's groups' keys (the searching
        ticket's CreatedAt, in this rank's group order) -> cp's totals and
        cp.positions, the global position of each of this rank's groups in the
        reference's order.  Two all-gathers and one all-reduce per pass; the
        positions are computed in C on the library's persistent host threads
        (mm_merge_positions_ex).  tie_ids(): this rank's searching ticket ids,
        asked for only when two ranks' keys tie (the ids then order the tied
        groups).  cp.local_stats gets the merge's split: the counts'
        all-gather, which waits for the slowest rank's pass (merge_wait_ms),
        the other collectives + copies (merge_comm_ms) and the C merge
        (merge_c_ms)."""
        import time

        import torch
        t0 = time.perf_counter()
        ng = len(keys)
        # processDefault's groups ascend by key; an override's choice may not.
        # Each rank checks its own, and the flag travels with the counts, so
        # no rank re-reads the whole matrix to find out.
        asc = 1 if ng < 2 or bool(np.all(keys[1:] >= keys[:-1])) else 0
        # one all-gather of (groups, matched tickets, presences, ascending)
        hdr = [self._t(np.zeros(4, dtype=np.int64)) for _ in range(self.world)]
        self.dist.all_gather(hdr, self._t(np.array([ng, tickets, pres, asc], dtype=np.int64)))
        hdr = np.stack([self._host(h) for h in hdr])
        t_hdr = time.perf_counter()  # the first collective after the pass: it also absorbs the ranks' skew
        counts = np.ascontiguousarray(hdr[:, 0].astype(np.int32))
        cp.n_groups, cp.matched_tickets, cp.matched_presences = (int(x) for x in hdr[:, :3].sum(axis=0))
        sorted_all = int(hdr[:, 3].min()) == 1
        # one all-gather of the keys into a [world][m] matrix (padded to the
        # largest rank's count; one collective, one copy each way)
        m = max(int(counts.max()), 1)
        host_in, dev_in = self._staging("keys_in", m, torch.int64)
        host_out, dev_out = self._staging("keys_out", self.world * m, torch.int64)
        hin = host_in.numpy()
        hin[:ng] = keys
        hin[ng:m] = 0
        if self.comm_device is not None:
            dev_in[:m].copy_(host_in[:m], non_blocking=True)
            self.dist.all_gather_into_tensor(dev_out[:self.world * m], dev_in[:m])
            host_out[:self.world * m].copy_(dev_out[:self.world * m], non_blocking=False)
        else:
            self.dist.all_gather_into_tensor(dev_out[:self.world * m], dev_in[:m])
        allk = host_out.numpy()
        t1 = time.perf_counter()
        pos = np.zeros(max(ng, 1), dtype=np.int64)
        # the merge in C: when some rank's keys do not ascend (rc 2, the same
        # on every rank) the groups take the stable order by (key, rank, index)
        rc = router_lib().mm_merge_positions_ex(allk.ctypes.data, m, counts.ctypes.data, self.world, self.rank,
                                                1 if sorted_all else 0, pos.ctypes.data)
        cp.positions = pos[:ng]
        t2 = time.perf_counter()
        flag = self._t(np.array([1 if rc == 1 else 0], dtype=np.int32))
        self.dist.all_reduce(flag, op=self.dist.ReduceOp.MAX)
        if int(self._host(flag)[0]) and rc != 2:  # rare: the searching tickets' ids order the tied groups
            flat = np.concatenate([allk[r * m:r * m + int(counts[r])] for r in range(self.world)])
            self._order_ties(cp, flat, counts, tie_ids() if tie_ids is not None else [""] * ng)
        t3 = time.perf_counter()
        cp.local_stats["merge_wait_ms"] = 1e3 * (t_hdr - t0)
        cp.local_stats["merge_comm_ms"] = 1e3 * ((t1 - t_hdr) + (t3 - t2))
        cp.local_stats["merge_c_ms"] = 1e3 * (t2 - t1)

    def _override(self, out):
        """This rank's override hand-off -> (committed result, error).  An
        override that raises must not leave the pass open (later passes would
        fail with MM_ERR_STATE while the other ranks wait in the next
        collective): the candidates are committed as an empty choice, and
        Process tells every rank of the failure in one all-reduce."""
        err = None
        try:
            if self.override_commit is not None:
                res = self.override_commit(self.local, out)
            else:
                try:
                    cands = capi.Matchmaker._groups(out)
                finally:
                    self.local.lib.mm_free_matched(self.local.h, C.byref(out))
                chosen = self.local.override(cands) if self.local.override is not None else []
                res = self.local.commit_call(chosen)
        except Exception as e:  # close the pass with an empty choice
            err = e
            res = capi.mm_matched()
            rc = self.local.lib.mm_process_commit(self.local.h, None, None, 0, C.byref(res))
            if rc != capi.MM_OK:
                res = capi.mm_matched()
        return res, err

    def _order_ties(self, cp: ClusterPass, allk: np.ndarray, counts: np.ndarray, tie_ids):
        """Equal CreatedAt on two ranks: those groups are ordered by their
        searching ticket's id, the second key of the pinned active order."""
        gathered = [None] * self.world
        self.dist.all_gather_object(gathered, tie_ids)
        off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        allpos = sorted(((int(allk[off[r] + i]), gathered[r][i], r, i) for r in range(self.world)
                         for i in range(int(counts[r]))))
        for p, (_, _, r, i) in enumerate(allpos):
            if r == self.rank:
                cp.positions[i] = p

    def gather_groups(self, cp: ClusterPass) -> Optional[List[List[Tuple[str, int]]]]:
        """Rank 0: the merged group list in the reference's order (needs
        Process(keep_groups=True) on every rank)."""
        gathered = [None] * self.world
        self.dist.all_gather_object(gathered, (cp.local.groups if cp.local is not None else None,
                                               cp.positions.tolist()))
        if self.rank != 0:
            return None
        merged = [None] * cp.n_groups
        for groups, pos in gathered:
            for g, p in zip(groups, pos):
                merged[p] = g
        return merged

    # ---- mutators and state (routed or broadcast) ----
    def ticket_count(self) -> int:
        t = self._t(np.array([self.local.ticket_count()], dtype=np.int64))
        self.dist.all_reduce(t)
        return int(self._host(t)[0])

    def active_count(self) -> int:
        t = self._t(np.array([self.local.active_count()], dtype=np.int64))
        self.dist.all_reduce(t)
        return int(self._host(t)[0])

    def Extract(self) -> Optional[List[capi.Ticket]]:
        """Extract (matchmaker.go:684-723) of every rank, sorted by ticket (rank 0)."""
        gathered = [None] * self.world
        self.dist.all_gather_object(gathered, self.local.Extract())
        if self.rank != 0:
            return None
        return sorted((t for ts in gathered for t in ts), key=lambda t: t.ticket)

    # Mutators.  Every rank calls each of them (a collective), passing its own
    # request or None; the requests of all ranks are gathered and applied on
    # every rank in rank order — the rank holding a ticket removes it, the
    # others find nothing — so a caller may name a ticket that lives on any rank.
    def _gather(self, req):
        gathered = [None] * self.world
        self.dist.all_gather_object(gathered, req)
        return gathered

    def _targeted(self, fn, req) -> Optional[Exception]:
        """fn(local, *args) for every rank's request on every rank; a request
        succeeds when the rank holding its ticket succeeds.  Returns this
        rank's error (None: success or no request)."""
        reqs = self._gather(req)
        # per request r: st[r] = 1 when the rank holding it removed it,
        # st[world + r] = 1 when some rank failed on it otherwise.  Every rank
        # takes part in the all_reduce whatever happened locally (an
        # exception here would leave the others hanging in the collective); a
        # local failure is re-raised after it.
        st = np.zeros(2 * self.world, dtype=np.int32)
        local_exc = None
        for r, q in enumerate(reqs):
            if q is None:
                continue
            try:
                fn(self.local, *q)
                st[r] = 1
            except capi.ErrMatchmakerTicketNotFound:
                pass
            except Exception as e:  # noqa: BLE001 - re-raised below, after the collective
                st[self.world + r] = 1
                if local_exc is None:
                    local_exc = e
        t = self._t(st)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        if local_exc is not None:
            raise local_exc
        if req is None:
            return None
        h = self._host(t)
        if int(h[self.rank]):
            return None
        if int(h[self.world + self.rank]):
            return capi.MatchmakerError(f"request {req!r} failed on another rank")
        return capi.ErrMatchmakerTicketNotFound(req[-1])

    def Remove(self, tickets: Optional[Sequence[str]]):
        """Remove (matchmaker.go:972-1024) of ids that may live on any rank."""
        ids = [t for ts in self._gather(list(tickets or [])) for t in ts]
        if ids:
            self.local.Remove(ids)

    def RemoveSession(self, session_id: Optional[str], ticket: Optional[str] = None):
        """RemoveSession (matchmaker.go:725-767); ErrMatchmakerTicketNotFound
        unless the rank holding the ticket removed it."""
        err = self._targeted(lambda m, sid, tk: m.RemoveSession(sid, tk),
                             None if session_id is None else (session_id, ticket))
        if err is not None:
            raise err

    def RemoveParty(self, party_id: Optional[str], ticket: Optional[str] = None):
        """RemoveParty (matchmaker.go:830-870)."""
        err = self._targeted(lambda m, pid, tk: m.RemoveParty(pid, tk), None if party_id is None else (party_id, ticket))
        if err is not None:
            raise err

    def RemoveSessionAll(self, session_id: Optional[str]):
        """RemoveSessionAll (matchmaker.go:769-828): one session's tickets on every rank."""
        for sid in self._gather(session_id):
            if sid is not None:
                self.local.RemoveSessionAll(sid)

    def RemovePartyAll(self, party_id: Optional[str]):
        """RemovePartyAll (matchmaker.go:872-917)."""
        for pid in self._gather(party_id):
            if pid is not None:
                self.local.RemovePartyAll(pid)

    def RemoveAll(self, node: Optional[str]):
        """RemoveAll (matchmaker.go:919-970)."""
        for nd in self._gather(node):
            if nd is not None:
                self.local.RemoveAll(nd)

    def Add(self, ticket: Optional[capi.Ticket]) -> Optional[Exception]:
        """Add (matchmaker.go:443-565) of this rank's ticket (or None), routed
        to its pool's rank (a new pool goes to the least-loaded rank).
        Returns the caller's error (None: added).  MaxTickets is checked by
        the owning rank's handle against the tickets it holds: a session
        whose tickets sit in pools of different ranks is limited per rank.
        The exact node-wide check is the in-process front's (mm_create_multi,
        include/nakama_cluster.h), the handle a Go server drives."""
        reqs = self._gather(ticket)
        mine = capi._TicketPack([ticket] if ticket is not None else [])
        self._place_new_pools(route_keys(mine.arr, 1 if ticket is not None else 0, self.pool_fields))
        pack = capi._TicketPack([t for t in reqs if t is not None])
        keys = route_keys(pack.arr, sum(t is not None for t in reqs), self.pool_fields)
        own = self.owners(keys)
        err = None
        local_exc = None  # a failure that is not a matchmaker status: re-raised after every collective
        k = 0
        for r, t in enumerate(reqs):
            if t is None:
                continue
            e = None
            if own[k] < 0:
                e = capi.ErrMatchmakerUnsupportedQuery("query does not pin every pool field to the ticket's own value")
            elif own[k] == self.rank:
                try:
                    self.local.Add(t.presences, t.session_id, t.party_id, t.query, t.min_count, t.max_count,
                                   t.count_multiple, t.string_properties, t.numeric_properties, ticket=t.ticket,
                                   created_at=t.created_at)
                except capi.MatchmakerError as x:
                    e = x
                except Exception as x:  # noqa: BLE001 - the requester gets a MatchmakerError, this rank re-raises
                    e = capi.MatchmakerError(f"{type(x).__name__}: {x}")
                    if local_exc is None:
                        local_exc = x
            codes = [None] * self.world
            self.dist.all_gather_object(codes, None if e is None else (type(e).__name__, str(e)) if own[k] == self.rank or own[k] < 0 else None)
            src = own[k] if own[k] >= 0 else r
            got = codes[src]
            if r == self.rank and got is not None:
                cls = getattr(capi, got[0], capi.MatchmakerError)
                err = cls(got[1])
            k += 1
        if local_exc is not None:
            raise local_exc
        return err


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64))


class RowShardedMatchmaker:
    """The row-sharded mode (include/nakama_cluster.h): for queries that cross
    pools, every rank holds the whole ticket set and runs the same pass; each
    batch's searches are split into one block per rank and the blocks'
    results are exchanged in place before the (replicated) ordered replay, so
    every rank forms the reference's groups.  transport "rccl": the exchange
    runs inside the library as RCCL broadcasts between device buffers (xGMI);
    "host": through a gloo all-gather of host buffers (the one-GPU rehearsal:
    RCCL cannot put two ranks on one device); None: replicas only, no split.
    Every method is a collective."""

    def __init__(self, local: capi.Matchmaker, dist, transport: Optional[str] = "rccl"):
        self.local = local
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.transport = transport
        lib = router_lib()
        lib.mm_shard_rows.restype = C.c_int
        lib.mm_shard_rows.argtypes = [C.c_void_p, C.c_int32, C.c_int32, ALLGATHER_FN, C.c_void_p]
        lib.mm_shard_rows_rccl.restype = C.c_int
        lib.mm_shard_rows_rccl.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32]
        lib.mm_rccl_unique_id.restype = C.c_int
        lib.mm_rccl_unique_id.argtypes = [C.c_void_p, C.c_int32]
        self.gather_bytes = 0  # exchanged by this rank's host all-gathers (host transport)
        if transport == "rccl":
            uid = (C.c_uint8 * 128)()
            if self.rank == 0 and lib.mm_rccl_unique_id(uid, 128) != 0:
                raise capi.ErrDevice("ncclGetUniqueId failed")
            box = [bytes(uid) if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            buf = (C.c_uint8 * 128).from_buffer_copy(box[0])
            local._check(lib.mm_shard_rows_rccl(local.h, self.world, self.rank, buf, 128))
        elif transport == "host":
            self._fn = ALLGATHER_FN(self._allgather)
            local._check(lib.mm_shard_rows(local.h, self.world, self.rank, self._fn, None))
        # transport None: replicas only — every rank runs the whole pass itself
        # (the CPU tests of the replication plumbing, over the oracle)

    def _allgather(self, _ctx, buf, offsets) -> int:
        """mm_allgather_fn over gloo: fill every other rank's segment of buf."""
        import torch
        try:
            off = [offsets[i] for i in range(self.world + 1)]
            sizes = [off[q + 1] - off[q] for q in range(self.world)]
            m = max(max(sizes), 1)
            mine = np.zeros(m, dtype=np.uint8)
            n = sizes[self.rank]
            if n:
                C.memmove(mine.ctypes.data, buf + off[self.rank], n)
            outs = [torch.zeros(m, dtype=torch.uint8) for _ in range(self.world)]
            self.dist.all_gather(outs, torch.from_numpy(mine))
            for q in range(self.world):
                if q != self.rank and sizes[q]:
                    C.memmove(buf + off[q], outs[q].numpy().ctypes.data, sizes[q])
            self.gather_bytes += sum(sizes)
            return 0
        except Exception:
            return 1

    def Insert(self, tickets, n: int):
        """Insert of this rank's ingest batch, replicated: every rank inserts
        every rank's tickets, in rank order (identical stores)."""
        import torch
        buf = pack(tickets, np.arange(n, dtype=np.int32)) if n else np.zeros(0, dtype=np.uint8)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(self.world)]
        self.dist.all_gather(sizes, torch.tensor([len(buf)], dtype=torch.int64))
        sizes = [int(s.item()) for s in sizes]
        m = max(max(sizes), 1)
        pad = np.zeros(m, dtype=np.uint8)
        pad[:len(buf)] = buf
        outs = [torch.zeros(m, dtype=torch.uint8) for _ in range(self.world)]
        self.dist.all_gather(outs, torch.from_numpy(pad))
        for q in range(self.world):
            u = Unpacked(outs[q].numpy()[:sizes[q]])
            try:
                if u.n.value:
                    self.local._check(self.local.lib.mm_insert(self.local.h, u.tickets, u.n.value))
            finally:
                u.close()

    def Remove(self, tickets: Sequence[str]):
        gathered = [None] * self.world
        self.dist.all_gather_object(gathered, list(tickets))
        self.local.Remove([t for ts in gathered for t in ts])

    def Process(self) -> capi.ProcessResult:
        """The pass, searches split over the ranks; every rank returns the
        same groups (the reference's, in its order)."""
        return self.local.process_raw()

    def Extract(self):
        return self.local.Extract()
