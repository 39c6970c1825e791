"""Seeded synthetic ticket sets (tools/synth.cpp) for tests and bench.py.

The generator returns native mm_ticket arrays that are passed unchanged to
mm_insert of the HIP library or the CPU oracle, so both see identical inputs.
Configs 1..5 follow BASELINE.json configs[0..4] / SURVEY.md 8(d); config 6 is
a small mixed workload (parties, ranges, boosts, Min<Max, CountMultiple) for
parity tests.
"""
import ctypes as C
import os
import subprocess

from . import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "libmm_synth.so")
T0 = (1_700_000_000_000_000_000 // 1024) * 1024
SEEDS = {1: 0x5EED0001, 2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005, 6: 0x5EED0006, 8: 0x5EED0008, 9: 0x5EED0009, 11: 0x5EED0005, 12: 0x5EED0006, 13: 0x5EED0005, 14: 0x5EED0005}
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(ROOT, "tools", "synth.cpp")):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True)
        _lib = C.CDLL(SO)
        _lib.synth_make.restype = C.c_void_p
        _lib.synth_make.argtypes = [C.c_int, C.c_uint64, C.c_int64, C.c_int64, C.c_int64]
        _lib.synth_tickets.restype = C.POINTER(capi.mm_ticket)
        _lib.synth_tickets.argtypes = [C.c_void_p]
        _lib.synth_count.restype = C.c_int64
        _lib.synth_count.argtypes = [C.c_void_p]
        _lib.synth_presences.restype = C.c_int64
        _lib.synth_presences.argtypes = [C.c_void_p]
        _lib.synth_free.argtypes = [C.c_void_p]
        _lib.synth_make_pools.restype = C.c_void_p
        _lib.synth_make_pools.argtypes = [C.c_int, C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_uint64]
        _lib.synth_make_shard.restype = C.c_void_p
        _lib.synth_make_shard.argtypes = [C.c_int, C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int]
        _lib.synth_pool_of.restype = C.c_int
        _lib.synth_pool_of.argtypes = [C.c_int, C.c_uint64, C.c_uint64]
        _lib.synth_make_scaled.restype = C.c_void_p
        _lib.synth_make_scaled.argtypes = [C.c_int, C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int]
        _lib.synth_override_first_disjoint.restype = C.c_int32
        _lib.synth_override_first_disjoint.argtypes = [C.POINTER(C.c_int32), C.POINTER(capi.mm_entry_ref), C.c_int32,
                                                       C.POINTER(C.c_int32), C.POINTER(capi.mm_entry_ref)]
        _lib.synth_sha_new.restype = C.c_void_p
        _lib.synth_sha_new.argtypes = []
        _lib.synth_sha_bytes.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
        _lib.synth_sha_groups.restype = C.c_int64
        _lib.synth_sha_groups.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(capi.mm_entry_ref), C.c_int32]
        _lib.synth_sha_extract.argtypes = [C.c_void_p, C.POINTER(capi.mm_ticket), C.c_int32]
        _lib.synth_sha_final.argtypes = [C.c_void_p, C.c_char_p]
    return _lib


class Digest:
    """Streaming SHA-256 over the canonical text of group lists / post-pass
    states (tools/synth.cpp): groups as "<ticket>:<presence index>," per entry
    and "\\n" per group; a state as "<ticket>:<intervals>\\n" per remaining
    ticket in ascending id order.  hashlib over the same bytes agrees."""

    def __init__(self):
        self.h = lib().synth_sha_new()

    def groups_raw(self, out) -> int:
        """Adds an mm_matched's groups (native: no Python per entry)."""
        if out.n_groups == 0:
            return 0
        return lib().synth_sha_groups(self.h, out.group_offsets, out.entries, out.n_groups)

    def groups(self, groups) -> None:
        """Adds Python groups [[(ticket, pi), ...], ...]."""
        self.raw(groups_text(groups))

    def raw(self, b: bytes) -> None:
        lib().synth_sha_bytes(self.h, b, len(b))

    def extract_raw(self, mm: "capi.Matchmaker") -> int:
        """Adds mm's post-pass state (mm_extract through the C ABI); returns
        the remaining ticket count."""
        out = capi.mm_extract_list()
        mm._check(mm.lib.mm_extract(mm.h, C.byref(out)))
        try:
            lib().synth_sha_extract(self.h, out.tickets, out.n)
            return out.n
        finally:
            mm.lib.mm_free_extract(mm.h, C.byref(out))

    def hexdigest(self) -> str:
        buf = C.create_string_buffer(32)
        lib().synth_sha_final(self.h, buf)
        self.h = None
        return buf.raw.hex()


def groups_text(groups) -> bytes:
    return b"".join(b"".join(t.encode() + b":%d," % pi for t, pi in g) + b"\n" for g in groups)


N_POOLS = {3: 8, 4: 64}


def pool_of(config: int, i: int, seed: int = None) -> int:
    return lib().synth_pool_of(config, SEEDS.get(config, 1) if seed is None else seed, i)


class TicketSet:
    """Tickets [first, first+n) of a config; owns the native arrays."""

    def __init__(self, config: int, n: int, first: int = 0, seed: int = None, t0: int = T0, pool_mask: int = None,
                 shard: int = None, pool_groups: int = None):
        """pool_mask: keep only tickets of these pools (bit p = pool p) out of
        the n generated indices — a rank's shard of a pool-sharded set.
        shard: region values suffixed "-g<shard>" (configs 1-4): a disjoint
        copy of the config's pools.  pool_groups: ONE set whose regions carry
        "-g<h>", h drawn per ticket in [0, pool_groups) (configs 1-4): the
        config's pools times pool_groups, spread over every index range — the
        N-GPU weak-scaling workload the cluster front routes."""
        L = lib()
        self.config = config
        sd = SEEDS.get(config, 1) if seed is None else seed
        if pool_groups:
            self.h = L.synth_make_scaled(config, sd, first, n, t0, pool_groups)
        elif shard is not None:
            self.h = L.synth_make_shard(config, sd, first, n, t0, shard)
        elif pool_mask is None:
            self.h = L.synth_make(config, sd, first, n, t0)
        else:
            self.h = L.synth_make_pools(config, sd, first, n, t0, pool_mask)
        self.n = L.synth_count(self.h)
        self.presences = L.synth_presences(self.h)
        self.tickets = L.synth_tickets(self.h)

    def insert_into(self, mm: "capi.Matchmaker", chunk: int = 1 << 20):
        for off in range(0, self.n, chunk):
            cnt = min(chunk, self.n - off)
            ptr = C.cast(C.addressof(self.tickets.contents) + off * C.sizeof(capi.mm_ticket), C.POINTER(capi.mm_ticket))
            mm._check(mm.lib.mm_insert(mm.h, ptr, cnt))

    def ptr(self, off: int = 0):
        """mm_ticket* to ticket `off` of the native array."""
        return C.cast(C.addressof(self.tickets.contents) + off * C.sizeof(capi.mm_ticket), C.POINTER(capi.mm_ticket))

    def ticket_id(self, k: int) -> str:
        return self.tickets[k].ticket.decode()

    def close(self):
        if self.h:
            lib().synth_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def override_commit(mm: "capi.Matchmaker", out, times=None) -> "capi.mm_matched":
    """The bench's override step on a candidate result `out` (freed here): the
    native first-disjoint override (tools/synth.cpp) picks groups, and
    mm_process_commit hands them back.  Returns the commit's result (free it
    with the library's mm_free_matched).  times: a dict that receives the
    override's and the commit's milliseconds."""
    import time
    import numpy as np
    t0 = time.perf_counter()
    n = out.n_groups
    ne = out.n_entries
    # output room for every candidate, left uninitialised (numpy.empty: only
    # the pages the kept groups are written to get touched; a ctypes array
    # would zero-fill gigabytes)
    offs_buf = np.empty(n + 1, dtype=np.int32)
    ents_buf = np.empty(max(1, ne) * C.sizeof(capi.mm_entry_ref), dtype=np.uint8)
    offs = offs_buf.ctypes.data_as(C.POINTER(C.c_int32))
    ents = ents_buf.ctypes.data_as(C.POINTER(capi.mm_entry_ref))
    kept = lib().synth_override_first_disjoint(out.group_offsets, out.entries, n, offs, ents)
    t1 = time.perf_counter()
    res = capi.mm_matched()
    try:  # the kept entries point into the candidate result: it goes back after the commit
        mm._check(mm.lib.mm_process_commit(mm.h, offs, ents, kept, C.byref(res)))
    finally:
        mm.lib.mm_free_matched(mm.h, C.byref(out))
    if times is not None:
        times["override_ms"] = 1e3 * (t1 - t0)
        times["commit_ms"] = 1e3 * (time.perf_counter() - t1)
    return res
