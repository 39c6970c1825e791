"""Shared test harness: drives any library exporting include/nakama_mm.h.

Scenario runner for the known-answer fixtures (tests/golden/known_answer.json)
and the seeded synthetic workloads of SURVEY.md 8(d) (tools/workloads.py).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nakama_amd import capi  # noqa: E402

ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle_mm.so")
PRODUCT_SO = os.path.join(ROOT, "nakama_amd", "libnakama_mm.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def build_oracle():
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < max(
            os.path.getmtime(os.path.join(ROOT, "oracle", f)) for f in ("mm_oracle.cpp", "go_compat.h", "go_regexp.h", "unicode_ref.h")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_oracle_lib = None


def oracle_lib():
    global _oracle_lib
    if _oracle_lib is None:
        build_oracle()
        _oracle_lib = capi.load_library(ORACLE_SO)
    return _oracle_lib


def load_known_answer():
    with open(os.path.join(GOLDEN, "known_answer.json")) as f:
        return json.load(f)


def run_scenario(lib, sc, T0, step):
    """Runs one fixture scenario; returns (process_results, errors_seen)."""
    cfg = sc["config"]
    mm = capi.Matchmaker(lib, max_tickets=cfg.get("max_tickets", 3), max_intervals=cfg.get("max_intervals", 2),
                         rev_precision=cfg.get("rev_precision", False))
    results = []
    errors = []
    i = 0
    try:
        for op in sc["ops"]:
            if op["op"] == "add":
                pres = [capi.Presence(p["user_id"], p["session_id"], p["username"], p["node"]) for p in op["presences"]]
                err = None
                try:
                    mm.Add(pres, op["session_id"], op["party_id"], op["query"], op["min_count"], op["max_count"],
                           op["count_multiple"], op["string_properties"], op["numeric_properties"],
                           ticket=op["ticket"], created_at=T0 + step * i)
                except capi.MatchmakerError as e:
                    err = type(e).__name__
                errors.append((op["ticket"], err, op.get("expect_error")))
                i += 1
            elif op["op"] == "remove_session":
                mm.RemoveSession(op["session_id"], op["ticket"])
            elif op["op"] == "process":
                results.append(mm.Process())
        extract = mm.Extract()
    finally:
        mm.close()
    return results, errors, extract


def search_case_hit(lib, case, T0):
    """One single-document search of a `search_cases` fixture: the document is a
    ticket with Query "*" (Min=Max=2) and the case's string properties; the query
    runs as the search of a second ticket (no properties).  Returns whether the
    document is among the hits and the hit list."""
    mm = capi.Matchmaker(lib, max_intervals=5)
    try:
        mm.Add([capi.Presence("u1", "sid1", "u1", "n")], "sid1", "", "*", 2, 2, 1, case["doc"], {},
               ticket="ticket1", created_at=T0)
        mm.Add([capi.Presence("u2", "sid2", "u2", "n")], "sid2", "", case["query"], 2, 2, 1, {}, {},
               ticket="searcher", created_at=T0 + 1024)
        hits = mm.debug_hits("searcher")
    finally:
        mm.close()
    return "ticket1" in [h for h, _ in hits], hits


def term_match(lib, kind, pattern, fuzziness, term):
    """mm_debug_term_match -> [matched, boost] or "search_error" / "unsupported"."""
    import ctypes
    b = ctypes.c_double(0.0)
    rc = lib.mm_debug_term_match(kind, pattern.encode("utf-8", "surrogateescape"), fuzziness,
                                 term.encode("utf-8", "surrogateescape"), ctypes.byref(b))
    if rc == -1:
        return "search_error"
    if rc == -2:
        return "unsupported"
    return [rc, b.value if rc == 1 else 0]


CUSTOM_POOLS = {"a": 64, "b": 65, "c": 63, "d": 5}  # filtered hits per row: 63, 64, 62, 4


def custom_pool_candidates(lib, pools=CUSTOM_POOLS):
    """processCustom over interleaved pools of solo tickets, query
    "+properties.k:<own pool>", Min=2 Max=3: a row of a pool of n tickets has
    n-1 filtered hits.  combineIndexes loops `combinationBits < (1 << length)`
    over Go ints (server/matchmaker_process.go:588), so a row with 63 hits
    (1 << 63 is negative) or 64 (1 << 64 is 0) yields no candidate, while a
    row with 62 yields every 2-subset (1-subsets reach hitCount 2 < MaxCount
    with Intervals <= MaxIntervals and are rejected, :496).  Returns (the
    candidate list the override received, ticket -> pool)."""
    order = [(p, k) for p, n in pools.items() for k in range(n)]
    order.sort(key=lambda pk: ((pk[1] * 7919 + ord(pk[0]) * 104729) % 1009, pk[0], pk[1]))  # interleave the pools
    seen, pool_of = [], {}
    mm = capi.Matchmaker(lib, override=lambda c: (seen.append([list(g) for g in c]), [])[1], max_intervals=5)
    try:
        for i, (p, k) in enumerate(order):
            t = f"t-{p}-{k:03d}"
            pool_of[t] = p
            mm.Add([capi.Presence(f"u{i}", f"s{i}", f"u{i}", "n")], f"s{i}", "", f"+properties.k:{p}", 2, 3, 1,
                   {"k": p}, {}, ticket=t, created_at=1_700_000_000_000_000_000 + 1024 * i)
        mm.Process()
    finally:
        mm.close()
    return (seen[0] if seen else []), pool_of


def matched_sessions(groups, sc):
    """Session ids of matched entries (the test's matchesSeen keys)."""
    sess = {}
    for op in sc["ops"]:
        if op["op"] == "add":
            sess[op["ticket"]] = [p["session_id"] for p in op["presences"]]
    out = set()
    for g in groups:
        for t, pi in g:
            out.add(sess[t][pi])
    return out
