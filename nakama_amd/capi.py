"""ctypes binding of the C ABI declared in include/nakama_mm.h.

The same binding drives any shared object that exports that ABI: the HIP
product (nakama_amd/libnakama_mm.so) and, in tests only, the CPU oracle
(oracle/liboracle_mm.so).  `Matchmaker` mirrors the reference's
`server.Matchmaker` interface (server/matchmaker.go:169-183): method names,
argument meaning and error behaviour (nakama-common sentinels,
runtime/runtime.go:180-186) follow the Go interface.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

MM_OK = 0


class MatchmakerError(Exception):
    code = -100


class ErrMatchmakerQueryInvalid(MatchmakerError):
    code = -1


class ErrMatchmakerDuplicateSession(MatchmakerError):
    code = -2


class ErrMatchmakerIndex(MatchmakerError):
    code = -3


class ErrMatchmakerDelete(MatchmakerError):
    code = -4


class ErrMatchmakerNotAvailable(MatchmakerError):
    code = -5


class ErrMatchmakerTooManyTickets(MatchmakerError):
    code = -6


class ErrMatchmakerTicketNotFound(MatchmakerError):
    code = -7


class ErrMatchmakerUnsupportedQuery(ErrMatchmakerQueryInvalid):
    code = -8


class ErrDevice(MatchmakerError):
    code = -9


class ErrArgument(MatchmakerError):
    code = -10


class ErrState(MatchmakerError):
    code = -11


_ERRS = {c.code: c for c in (ErrMatchmakerQueryInvalid, ErrMatchmakerDuplicateSession, ErrMatchmakerIndex,
                             ErrMatchmakerDelete, ErrMatchmakerNotAvailable, ErrMatchmakerTooManyTickets,
                             ErrMatchmakerTicketNotFound, ErrMatchmakerUnsupportedQuery, ErrDevice, ErrArgument,
                             ErrState)}


def _b(s: Optional[str]) -> Optional[bytes]:
    return None if s is None else s.encode("utf-8")


class mm_config(C.Structure):
    _fields_ = [("max_tickets", C.c_int32), ("interval_sec", C.c_int32), ("max_intervals", C.c_int32),
                ("rev_precision", C.c_int32), ("rev_threshold", C.c_int32), ("override_enabled", C.c_int32),
                ("device", C.c_int32), ("node", C.c_char_p)]


class mm_presence(C.Structure):
    _fields_ = [("user_id", C.c_char_p), ("session_id", C.c_char_p), ("username", C.c_char_p),
                ("node", C.c_char_p)]


class mm_str_prop(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p)]


class mm_num_prop(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_double)]


class mm_ticket(C.Structure):
    _fields_ = [("ticket", C.c_char_p), ("session_id", C.c_char_p), ("party_id", C.c_char_p),
                ("query", C.c_char_p), ("min_count", C.c_int32), ("max_count", C.c_int32),
                ("count_multiple", C.c_int32), ("intervals", C.c_int32), ("created_at", C.c_int64),
                ("node", C.c_char_p), ("presences", C.POINTER(mm_presence)), ("n_presences", C.c_int32),
                ("str_props", C.POINTER(mm_str_prop)), ("n_str_props", C.c_int32),
                ("num_props", C.POINTER(mm_num_prop)), ("n_num_props", C.c_int32)]


class mm_entry_ref(C.Structure):
    _fields_ = [("ticket", C.c_char_p), ("presence_index", C.c_int32), ("reserved", C.c_int32)]


class mm_matched(C.Structure):
    _fields_ = [("n_groups", C.c_int32), ("n_entries", C.c_int32), ("group_offsets", C.POINTER(C.c_int32)),
                ("entries", C.POINTER(mm_entry_ref)), ("is_candidates", C.c_int32), ("n_expired", C.c_int32),
                ("pass_ms", C.c_double), ("eval_ms", C.c_double), ("pair_evals", C.c_int64),
                ("reserved2", C.c_int64), ("eval_bytes", C.c_int64), ("eval_launches", C.c_int32),
                ("n_batches", C.c_int32), ("eval_kernel", C.c_int32), ("full_lists", C.c_int32),
                ("group_created", C.POINTER(C.c_int64)), ("pairs_decided", C.c_int64)]


class mm_extract_list(C.Structure):
    _fields_ = [("n", C.c_int32), ("tickets", C.POINTER(mm_ticket))]


class mm_str_list(C.Structure):
    _fields_ = [("n", C.c_int32), ("items", C.POINTER(C.c_char_p))]


PASS_HOOK = C.CFUNCTYPE(None, C.c_void_p)
# mm_deliver_fn(ctx, matched, pass_seq) (include/nakama_mm.h, pipelined delivery)
DELIVER_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int64)

# mm_sub_api (include/nakama_cluster.h): the entry points a multi handle
# drives its sub-handles through, in declaration order -> exported symbol
SUB_API = (("create", "mm_create"), ("destroy", "mm_destroy"), ("pause", "mm_pause"), ("resume", "mm_resume"),
           ("stop", "mm_stop"), ("last_error", "mm_last_error"), ("add", "mm_add"), ("insert", "mm_insert"),
           ("extract", "mm_extract"), ("free_extract", "mm_free_extract"), ("remove_session", "mm_remove_session"),
           ("remove_session_all", "mm_remove_session_all"), ("remove_party", "mm_remove_party"),
           ("remove_party_all", "mm_remove_party_all"), ("remove_all", "mm_remove_all"), ("remove", "mm_remove"),
           ("process", "mm_process"), ("process_commit", "mm_process_commit"), ("free_matched", "mm_free_matched"),
           ("ticket_count", "mm_ticket_count"), ("active_count", "mm_active_count"),
           ("drain_removed", "mm_drain_removed"), ("free_str_list", "mm_free_str_list"),
           ("debug_hits", "mm_debug_hits"), ("debug_set_pass_hook", "mm_debug_set_pass_hook"),
           ("session_ticket_count", "mm_session_ticket_count"), ("party_ticket_count", "mm_party_ticket_count"),
           ("find_tickets", "mm_find_tickets"))


class mm_sub_api(C.Structure):
    _fields_ = [(f, C.c_void_p) for f, _ in SUB_API]


def sub_api(lib: C.CDLL) -> mm_sub_api:
    """The mm_sub_api table of a library exporting nakama_mm.h (e.g. the oracle)."""
    return mm_sub_api(*[C.cast(getattr(lib, sym), C.c_void_p) for _, sym in SUB_API])


MM_MULTI_POOLS, MM_MULTI_ROWS = 0, 1
MM_MULTI_AUTO, MM_MULTI_HOST, MM_MULTI_RCCL = 0, 1, 2


class mm_multi_config(C.Structure):
    _fields_ = [("devices", C.POINTER(C.c_int32)), ("n_devices", C.c_int32), ("mode", C.c_int32),
                ("pool_fields", C.POINTER(C.c_char_p)), ("n_pool_fields", C.c_int32), ("transport", C.c_int32),
                ("api", C.POINTER(mm_sub_api))]


EXPORTED_SYMBOLS = (
    "mm_create", "mm_destroy", "mm_pause", "mm_resume", "mm_stop", "mm_last_error", "mm_abi_version",
    "mm_backend_name", "mm_add", "mm_insert", "mm_extract", "mm_free_extract", "mm_remove_session",
    "mm_remove_session_all", "mm_remove_party", "mm_remove_party_all", "mm_remove_all", "mm_remove",
    "mm_process", "mm_process_commit", "mm_free_matched", "mm_ticket_count", "mm_active_count",
    "mm_debug_hits", "mm_debug_compile", "mm_debug_term_match", "mm_debug_group_indexes",
    "mm_drain_removed", "mm_free_str_list", "mm_debug_set_pass_hook", "mm_session_ticket_count",
    "mm_party_ticket_count", "mm_find_tickets", "mm_set_delivery", "mm_process_deliver",
    "mm_process_commit_deliver", "mm_delivery_flush",
)


_counter = None


def _count_tickets(out: "mm_matched") -> int:
    """Matched tickets of a result: mm_count_tickets of the product library
    (host threads; any library's mm_matched), numpy when it is not built."""
    global _counter
    if _counter is None:
        so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnakama_mm.so")
        try:
            lib = C.CDLL(so, mode=C.RTLD_LOCAL)
            lib.mm_count_tickets.restype = C.c_int64
            lib.mm_count_tickets.argtypes = [C.c_void_p]
            _counter = lib.mm_count_tickets
        except OSError:
            _counter = False
    if _counter:
        return int(_counter(C.addressof(out)))
    import numpy as np
    raw = (C.c_char * (out.n_entries * C.sizeof(mm_entry_ref))).from_address(C.addressof(out.entries.contents))
    return int(np.count_nonzero(np.frombuffer(raw, dtype=np.int32).reshape(-1, 4)[:, 2] == 0))


def load_library(path: str) -> C.CDLL:
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    lib = C.CDLL(path, mode=C.RTLD_LOCAL)
    vp = C.c_void_p
    sig = {
        "mm_create": (vp, [C.POINTER(mm_config)]),
        "mm_destroy": (None, [vp]),
        "mm_pause": (None, [vp]),
        "mm_resume": (None, [vp]),
        "mm_stop": (None, [vp]),
        "mm_last_error": (C.c_char_p, [vp]),
        "mm_abi_version": (C.c_int, []),
        "mm_backend_name": (C.c_char_p, []),
        "mm_add": (C.c_int, [vp, C.POINTER(mm_ticket)]),
        "mm_insert": (C.c_int, [vp, C.POINTER(mm_ticket), C.c_int32]),
        "mm_extract": (C.c_int, [vp, C.POINTER(mm_extract_list)]),
        "mm_free_extract": (None, [vp, C.POINTER(mm_extract_list)]),
        "mm_remove_session": (C.c_int, [vp, C.c_char_p, C.c_char_p]),
        "mm_remove_session_all": (C.c_int, [vp, C.c_char_p]),
        "mm_remove_party": (C.c_int, [vp, C.c_char_p, C.c_char_p]),
        "mm_remove_party_all": (C.c_int, [vp, C.c_char_p]),
        "mm_remove_all": (C.c_int, [vp, C.c_char_p]),
        "mm_remove": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_int32]),
        "mm_process": (C.c_int, [vp, C.POINTER(mm_matched)]),
        "mm_process_commit": (C.c_int, [vp, C.POINTER(C.c_int32), C.POINTER(mm_entry_ref), C.c_int32,
                                        C.POINTER(mm_matched)]),
        "mm_free_matched": (None, [vp, C.POINTER(mm_matched)]),
        "mm_ticket_count": (C.c_int32, [vp]),
        "mm_active_count": (C.c_int32, [vp]),
        "mm_debug_hits": (C.c_int32, [vp, C.c_char_p, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.c_int32]),
        "mm_debug_compile": (C.c_int, [C.c_char_p]),
        "mm_drain_removed": (C.c_int, [vp, C.POINTER(mm_str_list)]),
        "mm_free_str_list": (None, [vp, C.POINTER(mm_str_list)]),
        "mm_debug_set_pass_hook": (None, [vp, PASS_HOOK, vp]),
        "mm_session_ticket_count": (C.c_int32, [vp, C.c_char_p]),
        "mm_party_ticket_count": (C.c_int32, [vp, C.c_char_p]),
        "mm_find_tickets": (C.c_int32, [vp, C.POINTER(C.c_char_p), C.c_int32, C.POINTER(C.c_uint8)]),
        "mm_debug_term_match": (C.c_int, [C.c_int32, C.c_char_p, C.c_int32, C.c_char_p, C.POINTER(C.c_double)]),
        "mm_debug_group_indexes": (C.c_int32, [C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_int32, C.c_int32,
                                               C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                               C.c_int32]),
        "mm_set_delivery": (C.c_int, [vp, DELIVER_FN, vp, C.c_int32]),
        "mm_process_deliver": (C.c_int, [vp, C.POINTER(mm_matched)]),
        "mm_process_commit_deliver": (C.c_int, [vp, C.POINTER(C.c_int32), C.POINTER(mm_entry_ref), C.c_int32,
                                                C.POINTER(mm_matched)]),
        "mm_delivery_flush": (C.c_int, [vp]),
    }
    if hasattr(lib, "mm_create_multi"):  # the product: one handle over several devices (nakama_cluster.h)
        sig["mm_create_multi"] = (vp, [C.POINTER(mm_config), C.POINTER(mm_multi_config)])
        sig["mm_multi_info"] = (C.c_int32, [vp, C.c_int32])
        sig["mm_device_numa_node"] = (C.c_int32, [C.c_int32])
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


@dataclass
class Presence:
    """MatchmakerPresence (server/matchmaker.go:32-38)."""
    user_id: str
    session_id: str
    username: str = ""
    node: str = ""


@dataclass
class Ticket:
    """MatchmakerExtract (server/matchmaker.go:110-125) / Add arguments."""
    ticket: str
    presences: List[Presence]
    session_id: str = ""
    party_id: str = ""
    query: str = "*"
    min_count: int = 2
    max_count: int = 2
    count_multiple: int = 1
    string_properties: Dict[str, str] = field(default_factory=dict)
    numeric_properties: Dict[str, float] = field(default_factory=dict)
    created_at: int = 0
    intervals: int = 0
    node: str = ""


@dataclass
class ProcessResult:
    groups: List[List[Tuple[str, int]]]
    is_candidates: bool
    n_expired: int
    pass_ms: float
    eval_ms: float
    pair_evals: int
    eval_bytes: int = 0
    eval_launches: int = 0
    n_batches: int = 0
    eval_kernel: int = 0  # 0 search_kernel, 1 scan_kernel, 2 mscan_kernel, 3 rsmall_kernel, 4 mscan_hash_kernel, 5 rpack_kernel, 6 rsrc_merge_kernel, 7 rsrc_tile_kernel
    full_lists: int = 0   # variable-score searches run as host-sorted full lists
    pairs_decided: int = 0  # (row, candidate) pairs decided: rows that searched x their search's source


class _TicketPack:
    """Keeps the ctypes buffers of a batch of tickets alive for one call."""

    def __init__(self, tickets: Sequence[Ticket]):
        self.keep = []
        self.arr = (mm_ticket * max(1, len(tickets)))()
        for i, t in enumerate(tickets):
            ps = (mm_presence * max(1, len(t.presences)))()
            for k, p in enumerate(t.presences):
                ps[k] = mm_presence(_b(p.user_id), _b(p.session_id), _b(p.username), _b(p.node))
            sp = (mm_str_prop * max(1, len(t.string_properties)))()
            for k, (kk, vv) in enumerate(t.string_properties.items()):
                sp[k] = mm_str_prop(_b(kk), _b(vv))
            npp = (mm_num_prop * max(1, len(t.numeric_properties)))()
            for k, (kk, vv) in enumerate(t.numeric_properties.items()):
                npp[k] = mm_num_prop(_b(kk), float(vv))
            self.keep += [ps, sp, npp]
            self.arr[i] = mm_ticket(_b(t.ticket), _b(t.session_id), _b(t.party_id), _b(t.query), t.min_count,
                                    t.max_count, t.count_multiple, t.intervals, t.created_at, _b(t.node), ps,
                                    len(t.presences), sp, len(t.string_properties), npp,
                                    len(t.numeric_properties))


class Matchmaker:
    """The `server.Matchmaker` interface over one C-ABI implementation.

    Add/Insert/Extract/Remove*/Process/Pause/Resume/Stop keep the Go names
    (server/matchmaker.go:169-183).  `OnMatchedEntries` registers a callback
    invoked with the matched groups after each default-path Process, as
    LocalMatchmaker does (matchmaker.go:437-439); delivery (JWT, router) is the
    host's concern and is not modelled.
    """

    def __init__(self, lib: C.CDLL, *, max_tickets: int = 3, interval_sec: int = 15, max_intervals: int = 2,
                 rev_precision: bool = False, rev_threshold: int = 1, override=None, device: int = 0,
                 node: str = "node1", multi: Optional[dict] = None):
        """multi: one handle over several sub-handles (mm_create_multi,
        include/nakama_cluster.h): dict(devices=[...], mode=MM_MULTI_POOLS |
        MM_MULTI_ROWS, pool_fields=[...], transport=MM_MULTI_AUTO, sub_lib=None
        (this library) or another library exporting nakama_mm.h)."""
        self.lib = lib
        self._node_b = _b(node)
        cfg = mm_config(max_tickets, interval_sec, max_intervals, int(bool(rev_precision)), rev_threshold,
                        int(override is not None), device, self._node_b)
        if multi is None:
            self.h = lib.mm_create(C.byref(cfg))
        else:
            devs = list(multi.get("devices", [device]))
            fields = [f.encode() for f in multi.get("pool_fields", ())]
            self._multi_keep = [(C.c_int32 * len(devs))(*devs), (C.c_char_p * max(1, len(fields)))(*fields)]
            api = None
            if multi.get("sub_lib") is not None:
                self._multi_keep.append(sub_api(multi["sub_lib"]))
                api = C.pointer(self._multi_keep[-1])
            mc = mm_multi_config(self._multi_keep[0], len(devs), multi.get("mode", MM_MULTI_POOLS),
                                 self._multi_keep[1], len(fields), multi.get("transport", MM_MULTI_AUTO), api)
            self.h = lib.mm_create_multi(C.byref(cfg), C.byref(mc))
        if not self.h:
            raise ErrDevice((lib.mm_last_error(None) or b"mm_create failed").decode("utf-8", "replace"))
        self.override = override
        self._matched_fn = None
        self.node = node

    def close(self):
        if self.h:
            self.lib.mm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != MM_OK:
            cls = _ERRS.get(rc, MatchmakerError)
            raise cls(self.lib.mm_last_error(self.h).decode("utf-8", "replace") if self.h else str(rc))

    # lifecycle
    def Pause(self):
        self.lib.mm_pause(self.h)

    def Resume(self):
        self.lib.mm_resume(self.h)

    def Stop(self):
        self.lib.mm_stop(self.h)

    def OnMatchedEntries(self, fn):
        self._matched_fn = fn

    # mutators
    def Add(self, presences: Sequence[Presence], session_id: str, party_id: str, query: str, min_count: int,
            max_count: int, count_multiple: int, string_properties: Dict[str, str],
            numeric_properties: Dict[str, float], *, ticket: str, created_at: int) -> Tuple[str, int]:
        """Add (matchmaker.go:443).  The Go shim generates ticket (UUIDv4) and
        created_at (time.Now().UnixNano()) itself; here they are arguments so
        tests can pin them."""
        t = Ticket(ticket=ticket, presences=list(presences), session_id=session_id, party_id=party_id, query=query,
                   min_count=min_count, max_count=max_count, count_multiple=count_multiple,
                   string_properties=dict(string_properties), numeric_properties=dict(numeric_properties),
                   created_at=created_at)
        pack = _TicketPack([t])
        self._check(self.lib.mm_add(self.h, pack.arr))
        return ticket, created_at

    def Insert(self, extracts: Sequence[Ticket]):
        if not extracts:
            return
        pack = _TicketPack(extracts)
        self._check(self.lib.mm_insert(self.h, pack.arr, len(extracts)))

    def Extract(self) -> List[Ticket]:
        out = mm_extract_list()
        self._check(self.lib.mm_extract(self.h, C.byref(out)))
        res = []
        try:
            for i in range(out.n):
                t = out.tickets[i]
                d = lambda x: x.decode("utf-8") if x is not None else ""
                res.append(Ticket(
                    ticket=d(t.ticket), session_id=d(t.session_id), party_id=d(t.party_id), query=d(t.query),
                    min_count=t.min_count, max_count=t.max_count, count_multiple=t.count_multiple,
                    intervals=t.intervals, created_at=t.created_at, node=d(t.node),
                    presences=[Presence(d(t.presences[k].user_id), d(t.presences[k].session_id),
                                        d(t.presences[k].username), d(t.presences[k].node))
                               for k in range(t.n_presences)],
                    string_properties={d(t.str_props[k].key): d(t.str_props[k].value) for k in range(t.n_str_props)},
                    numeric_properties={d(t.num_props[k].key): t.num_props[k].value for k in range(t.n_num_props)},
                ))
        finally:
            self.lib.mm_free_extract(self.h, C.byref(out))
        res.sort(key=lambda t: t.ticket)
        return res

    def RemoveSession(self, session_id: str, ticket: str):
        self._check(self.lib.mm_remove_session(self.h, _b(session_id), _b(ticket)))

    def RemoveSessionAll(self, session_id: str):
        self._check(self.lib.mm_remove_session_all(self.h, _b(session_id)))

    def RemoveParty(self, party_id: str, ticket: str):
        self._check(self.lib.mm_remove_party(self.h, _b(party_id), _b(ticket)))

    def RemovePartyAll(self, party_id: str):
        self._check(self.lib.mm_remove_party_all(self.h, _b(party_id)))

    def RemoveAll(self, node: str):
        self._check(self.lib.mm_remove_all(self.h, _b(node)))

    def Remove(self, tickets: Sequence[str]):
        arr = (C.c_char_p * max(1, len(tickets)))(*[_b(t) for t in tickets])
        self._check(self.lib.mm_remove(self.h, arr, len(tickets)))

    # the interval pass
    @staticmethod
    def _groups(out: mm_matched) -> List[List[Tuple[str, int]]]:
        groups = []
        for g in range(out.n_groups):
            lo, hi = out.group_offsets[g], out.group_offsets[g + 1]
            groups.append([(out.entries[k].ticket.decode("utf-8"), out.entries[k].presence_index)
                           for k in range(lo, hi)])
        return groups

    def process_raw(self) -> ProcessResult:
        out = mm_matched()
        self._check(self.lib.mm_process(self.h, C.byref(out)))
        try:
            res = ProcessResult(self._groups(out), bool(out.is_candidates), out.n_expired, out.pass_ms, out.eval_ms,
                                out.pair_evals, out.eval_bytes, out.eval_launches, out.n_batches, out.eval_kernel,
                                out.full_lists, out.pairs_decided)
        finally:
            self.lib.mm_free_matched(self.h, C.byref(out))
        return res

    def process_call(self):
        """One mm_process call, nothing else: returns the library-owned result
        (pass it to process_summary, which frees it).  bench.py times exactly
        this call."""
        out = mm_matched()
        self._check(self.lib.mm_process(self.h, C.byref(out)))
        return out

    @staticmethod
    def summary_counts(out):
        """(n_groups, matched tickets, matched presences, ProcessResult without
        the groups) of a process_call result (not freed)."""
        n = out.n_entries
        tickets = _count_tickets(out) if n else 0
        res = ProcessResult([], bool(out.is_candidates), out.n_expired, out.pass_ms, out.eval_ms, out.pair_evals,
                            out.eval_bytes, out.eval_launches, out.n_batches, out.eval_kernel, out.full_lists,
                            out.pairs_decided)
        return out.n_groups, tickets, n, res

    def process_summary(self, out):
        """summary_counts of a process_call result; frees it."""
        try:
            return self.summary_counts(out)
        finally:
            self.lib.mm_free_matched(self.h, C.byref(out))

    def process_timed(self):
        """One mm_process call timed at the C boundary (no Python conversion of
        the groups inside the timed region).  Returns (seconds, n_groups,
        matched tickets, matched presences, ProcessResult-without-groups)."""
        import time
        t0 = time.perf_counter()
        out = self.process_call()
        dt = time.perf_counter() - t0
        return (dt,) + self.process_summary(out)

    def commit_call(self, groups: Sequence[Sequence[Tuple[str, int]]]):
        """mm_process_commit of (ticket, presence index) groups; returns the
        library-owned result (free it with the library's mm_free_matched)."""
        offs = [0]
        ents = []
        for g in groups:
            ents.extend(g)
            offs.append(len(ents))
        off_arr = (C.c_int32 * len(offs))(*offs)
        keep = [_b(t) for t, _ in ents]
        ent_arr = (mm_entry_ref * max(1, len(ents)))()
        for i, (t, pi) in enumerate(ents):
            ent_arr[i] = mm_entry_ref(keep[i], pi, 0)
        out = mm_matched()
        self._check(self.lib.mm_process_commit(self.h, off_arr, ent_arr, len(groups), C.byref(out)))
        return out

    def commit(self, groups: Sequence[Sequence[Tuple[str, int]]]) -> ProcessResult:
        offs = [0]
        ents = []
        for g in groups:
            for (t, pi) in g:
                ents.append((t, pi))
            offs.append(len(ents))
        off_arr = (C.c_int32 * len(offs))(*offs)
        keep = [_b(t) for t, _ in ents]
        ent_arr = (mm_entry_ref * max(1, len(ents)))()
        for i, (t, pi) in enumerate(ents):
            ent_arr[i] = mm_entry_ref(keep[i], pi, 0)
        out = mm_matched()
        self._check(self.lib.mm_process_commit(self.h, off_arr, ent_arr, len(groups), C.byref(out)))
        try:
            res = ProcessResult(self._groups(out), False, out.n_expired, out.pass_ms, out.eval_ms, out.pair_evals)
        finally:
            self.lib.mm_free_matched(self.h, C.byref(out))
        return res

    def Process(self) -> List[List[Tuple[str, int]]]:
        """Process (matchmaker.go:282).  Returns the matched groups as
        (ticket, presence index) lists; with an override registered the
        candidates go through `override(candidates) -> chosen` first
        (RuntimeMatchmakerOverrideFunction, runtime.go:212)."""
        r = self.process_raw()
        if r.is_candidates:
            chosen = self.override(r.groups) if self.override is not None else []
            r = self.commit(chosen)
        if r.groups and self._matched_fn is not None:
            self._matched_fn(r.groups)
        return r.groups

    # pipelined delivery (include/nakama_mm.h; matchmaker.go:374-440 behind the next pass)
    def set_delivery(self, fn, depth: int = 4):
        """fn(groups, pass_seq) is called on the library's delivery thread once
        per pass, in pass order, with the pass's matched groups; None stops
        the delivery after the queued results.  The ctypes trampoline is kept
        on the handle (the library holds a raw pointer to it)."""
        if fn is None:
            self._check(self.lib.mm_set_delivery(self.h, C.cast(None, DELIVER_FN), None, 0))
            self._deliver_cb = None
            return
        groups_of = self._groups

        def tramp(_ctx, matched, seq):
            fn(groups_of(C.cast(matched, C.POINTER(mm_matched)).contents), int(seq))

        cb = DELIVER_FN(tramp)
        self._check(self.lib.mm_set_delivery(self.h, cb, None, depth))
        self._deliver_cb = cb

    def process_deliver(self) -> ProcessResult:
        """One pass through mm_process_deliver: the groups go to the delivery
        callback; returns the counts (groups empty) — or, on the override
        path, the candidates in full (is_candidates), to be chosen and passed
        to commit_deliver."""
        out = mm_matched()
        self._check(self.lib.mm_process_deliver(self.h, C.byref(out)))
        if out.is_candidates:
            try:
                return ProcessResult(self._groups(out), True, out.n_expired, out.pass_ms, out.eval_ms, out.pair_evals,
                                     out.eval_bytes, out.eval_launches, out.n_batches, out.eval_kernel,
                                     out.full_lists, out.pairs_decided)
            finally:
                self.lib.mm_free_matched(self.h, C.byref(out))
        return ProcessResult([], False, out.n_expired, out.pass_ms, out.eval_ms, out.pair_evals, out.eval_bytes,
                             out.eval_launches, out.n_batches, out.eval_kernel, out.full_lists, out.pairs_decided)

    def commit_deliver(self, groups: Sequence[Sequence[Tuple[str, int]]]) -> int:
        """mm_process_commit_deliver of the override's choice; returns the
        committed group count (the groups go to the delivery callback)."""
        offs = [0]
        ents = []
        for g in groups:
            ents.extend(g)
            offs.append(len(ents))
        off_arr = (C.c_int32 * len(offs))(*offs)
        keep = [_b(t) for t, _ in ents]
        ent_arr = (mm_entry_ref * max(1, len(ents)))()
        for i, (t, pi) in enumerate(ents):
            ent_arr[i] = mm_entry_ref(keep[i], pi, 0)
        out = mm_matched()
        self._check(self.lib.mm_process_commit_deliver(self.h, off_arr, ent_arr, len(groups), C.byref(out)))
        return out.n_groups

    def delivery_flush(self):
        self._check(self.lib.mm_delivery_flush(self.h))

    def drain_removed(self) -> List[str]:
        """Tickets that left the matchmaker since the previous call (the first
        call starts the recording): what the Go shim drops from its delivery
        entries (include/nakama_mm.h, ABI 3)."""
        out = mm_str_list()
        self._check(self.lib.mm_drain_removed(self.h, C.byref(out)))
        try:
            return [out.items[i].decode("utf-8") for i in range(out.n)]
        finally:
            self.lib.mm_free_str_list(self.h, C.byref(out))

    def set_pass_hook(self, fn):
        """Test hook: fn() runs once per pass between the searches/replay and
        the post-pass finish, with the handle unlocked (mutators called from it
        are queued as concurrent ones).  None removes it."""
        self._hook = PASS_HOOK(lambda _ctx: fn()) if fn is not None else None
        self.lib.mm_debug_set_pass_hook(self.h, self._hook if fn is not None else PASS_HOOK(), None)

    # introspection
    def session_ticket_count(self, session_id: str) -> int:
        return int(self.lib.mm_session_ticket_count(self.h, _b(session_id)))

    def party_ticket_count(self, party_id: str) -> int:
        return int(self.lib.mm_party_ticket_count(self.h, _b(party_id)))

    def find_tickets(self, tickets: Sequence[str]) -> List[bool]:
        ids = (C.c_char_p * max(1, len(tickets)))(*[_b(t) for t in tickets])
        found = (C.c_uint8 * max(1, len(tickets)))()
        n = self.lib.mm_find_tickets(self.h, ids, len(tickets), found)
        if n < 0:
            self._check(n)
        return [bool(found[i]) for i in range(len(tickets))]

    def ticket_count(self) -> int:
        return self.lib.mm_ticket_count(self.h)

    def active_count(self) -> int:
        return self.lib.mm_active_count(self.h)

    def debug_hits(self, ticket: str, cap: int = 1 << 16) -> List[Tuple[str, float]]:
        tk = (C.c_char_p * cap)()
        sc = (C.c_double * cap)()
        n = self.lib.mm_debug_hits(self.h, _b(ticket), tk, sc, cap)
        if n < 0:
            raise ErrMatchmakerTicketNotFound(ticket)
        return [(tk[i].decode("utf-8"), sc[i]) for i in range(min(n, cap))]


def group_indexes(lib: C.CDLL, counts: Sequence[int], created: Sequence[int], required: int):
    """groupIndexes (matchmaker.go:132-167) through the library's debug entry."""
    n = len(counts)
    cap = 4096
    c_arr = (C.c_int32 * max(1, n))(*counts)
    t_arr = (C.c_int64 * max(1, n))(*created)
    g_off = (C.c_int32 * (cap + 1))()
    g_idx = (C.c_int32 * (cap * 8))()
    g_avg = (C.c_int64 * cap)()
    ng = lib.mm_debug_group_indexes(c_arr, t_arr, n, required, g_off, g_idx, g_avg, cap)
    out = []
    for g in range(ng):
        out.append(([g_idx[k] for k in range(g_off[g], g_off[g + 1])], g_avg[g]))
    return out
