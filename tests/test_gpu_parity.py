"""Parity of the HIP path with the CPU oracle (needs a gfx950 GPU).

Bar: bit-exact matched groups (ticket, presence index, entry order, group
order), identical post-pass state (remaining tickets, their Intervals, the
active set), identical hit lists (order) and scores (exact for the dyadic
boosts used here; the tolerance in the test is 1e-6 relative, as north_star
states) — all through the C ABI of include/nakama_mm.h.
"""
import math
import os
import re

import pytest

import harness
from nakama_amd import capi, synth

pytestmark = pytest.mark.gpu

KA = harness.load_known_answer()


def product_lib():
    import nakama_amd
    return nakama_amd.load_library()


def pair(cfg, **kw):
    return (capi.Matchmaker(product_lib(), **cfg, **kw), capi.Matchmaker(harness.oracle_lib(), **cfg, **kw))


@pytest.mark.parametrize("sc", KA["scenarios"], ids=[s["name"] for s in KA["scenarios"]])
def test_known_answer_gpu(sc):
    results, errors, extract = harness.run_scenario(product_lib(), sc, KA["T0"], KA["created_step"])
    for ticket, got, want in errors:
        assert got == want
    groups = [g for r in results for g in r]
    a = sc["assert"]
    sess = harness.matched_sessions(groups, sc)
    if "matched_sessions_count" in a:
        assert len(sess) == a["matched_sessions_count"], (sc["name"], groups)
    for s in a.get("matched_sessions_include", []):
        assert s in sess
    if sc["pinned_groups"] is not None:
        assert [[list(e) for e in g] for g in groups] == sc["pinned_groups"]
    # and the post-pass state equals the oracle's
    o_results, _, o_extract = harness.run_scenario(harness.oracle_lib(), sc, KA["T0"], KA["created_step"])
    assert results == o_results
    assert [(t.ticket, t.intervals) for t in extract] == [(t.ticket, t.intervals) for t in o_extract]


def state(mm):
    """Post-pass store state: every extracted field of every ticket (sessions,
    party, query, node, presences, properties, intervals) + the active count."""
    return mm.Extract(), mm.active_count()


# Oracle runs are memoised per workload: the kernel / host-path variants of a
# config compare the product against one oracle run (C1 10k is ~16 s of oracle).
_ORACLE_RUNS = {}


def _oracle_passes(config, n, passes, cfg):
    key = (config, n, passes, tuple(sorted(cfg.items())))
    if key not in _ORACLE_RUNS:
        ts = synth.TicketSet(config, n)
        orc = capi.Matchmaker(harness.oracle_lib(), **cfg)
        try:
            ts.insert_into(orc)
            _ORACLE_RUNS[key] = [(orc.Process(), state(orc)) for _ in range(passes)]
        finally:
            orc.close()
            ts.close()
    return _ORACLE_RUNS[key]


def run_passes(config, n, passes, cfg, extra=None):
    """Product passes against the (memoised) oracle's; returns the product's
    ProcessResults (groups + pass statistics)."""
    want = _oracle_passes(config, n, passes, cfg)
    ts = synth.TicketSet(config, n)
    gpu = capi.Matchmaker(product_lib(), **cfg)
    out = []
    try:
        ts.insert_into(gpu)
        for p in range(passes):
            r = gpu.process_raw()
            assert r.groups == want[p][0], f"config {config} pass {p}: groups differ (gpu {len(r.groups)} vs oracle {len(want[p][0])})"
            assert state(gpu) == want[p][1]
            if extra:
                extra(p, gpu)
            out.append(r)
        return out
    finally:
        gpu.close()
        ts.close()


# NKM_KERNEL routes a batch's constant-score searches to one query-eval
# kernel at any size (auto picks by size/coverage, which the small oracle
# workloads here never reach): every kernel is checked against the oracle.
# "mscan": the multi-signature scan as chosen by default — hashed
# (mscan_hash_kernel) past mscan_kernel's 16 signatures (C4's 64 pools) or
# when the scan order is the slot order (fresh sets: the contiguous mode);
# "mhash": hashed whenever the signatures allow it; "mscan16": never hashed
# (mscan_kernel; C4 then falls back to scan).
KERNELS = ["search", "scan", "mscan", "mscan16", "mhash"]


def set_kernel(monkeypatch, kernel):
    monkeypatch.setenv("NKM_KERNEL", "mscan" if kernel in ("mhash", "mscan16") else kernel)
    if kernel in ("mhash", "mscan16"):
        monkeypatch.setenv("NKM_MHASH", "1" if kernel == "mhash" else "2")


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("n", [1200, 10_000])
def test_c1_pool_query(kernel, n, monkeypatch):
    """C1 at its stated 10k (BASELINE configs[0]) on every query-eval kernel."""
    set_kernel(monkeypatch, kernel)
    run_passes(1, n, 2, dict(max_intervals=2))


def test_c2_skill_window_boosts():
    run_passes(2, 1500, 2, dict(max_intervals=2))


@pytest.mark.parametrize("fullvar", ["1", "0"])
def test_c2_region_lists_past_topk(fullvar, monkeypatch):
    """C2's shape at 10k: region posting lists of ~2,500 (past the 512-entry
    LDS top-K), ~1,000 skill-window signatures, so search_kernel<512>'s
    truncation, early exit at the score bound and batch restarts all run;
    NKM_FULLVAR=1 also sends re-searched rows through full lists.  (Top-tier
    lists and range batches off: they would keep rows from running off their
    lists.)"""
    monkeypatch.setenv("NKM_RANGE", "0")
    monkeypatch.setenv("NKM_TIER", "0")
    monkeypatch.setenv("NKM_FULLVAR", fullvar)
    rs = run_passes(2, 10_000, 2, dict(max_intervals=2))
    assert sum(r.n_batches for r in rs) > 2  # truncated lists restarted batches
    full = sum(r.full_lists for r in rs)
    assert (full > 0) if fullvar == "1" else (full == 0)


@pytest.mark.parametrize("mode", ["0", "2"])
@pytest.mark.parametrize("config,n,cfg", [(2, 10_000, dict(max_intervals=2)), (4, 3000, dict(max_intervals=2)),
                                          (5, 2000, dict(max_intervals=2, rev_precision=True, rev_threshold=0)),
                                          (7, 3000, dict(max_intervals=2))])
def test_hit_list_transfer_modes(config, n, cfg, mode, monkeypatch):
    """Hit lists back to the host as 16-B DHits (NKM_SLOTLISTS=0) and as slot
    ids for RevPrecision batches too (2; the default packs the others only),
    with the kernel forced to the chunked scan so chunked lists page."""
    monkeypatch.setenv("NKM_SLOTLISTS", mode)
    monkeypatch.setenv("NKM_KERNEL", "scan")
    run_passes(config, n, 2, cfg)


@pytest.mark.parametrize("config,n,cfg", [(2, 10_000, dict(max_intervals=2)), (2, 30_000, dict(max_intervals=2)),
                                          (9, 5000, dict(max_intervals=2)), (10, 3000, dict(max_intervals=2)),
                                          (6, 2000, dict(max_intervals=3)), (8, 2000, dict(max_intervals=3))])
@pytest.mark.parametrize("tier", ["1", "0"])
def test_top_tier_lists(config, n, cfg, tier, monkeypatch):
    """Variable-score searches as top-tier lists (search_kernel path 2: the
    hits scoring the query's top score, in source order — an exact prefix of
    the sorted hit list of any length) when every clause score sums exactly:
    C2's skill windows (boosts ^2), config 9 (no region must), wide queries
    and mixed workloads (non-dyadic boosts keep the LDS top-K).  Groups and
    state equal to the oracle; C2 at 30k needs no more than 3 batches.  (Range
    batches off: they take C2's rows otherwise.)"""
    monkeypatch.setenv("NKM_RANGE", "0")
    monkeypatch.setenv("NKM_TIER", tier)
    rs = run_passes(config, n, 2, cfg)
    if config == 2 and n == 30_000 and tier == "1":
        assert rs[0].n_batches <= 3, rs[0].n_batches


@pytest.mark.parametrize("par", ["1", "force"])
@pytest.mark.parametrize("config,n,passes,cfg", [(2, 1500, 2, dict(max_intervals=2)), (2, 10_000, 2, dict(max_intervals=2)),
                                                 (2, 30_000, 2, dict(max_intervals=2)), (15, 3000, 3, dict(max_intervals=3)),
                                                 (15, 12_000, 2, dict(max_intervals=2)), (16, 3000, 3, dict(max_intervals=3))])
def test_range_batches(config, n, passes, cfg, par, monkeypatch):
    """Range batches (mm_range.cpp, range_walk.h): every row a pool term plus
    numeric ranges on one field — C2's skill windows; config 15 adds parties,
    Min < Max, CountMultiple, Intervals, MUST_NOT and ^0.5 ranges and tickets
    whose skill is a keyword; 16 puts every ticket in one pool.  The pools'
    candidates are sorted on the device (rsrc_tile / rsrc_merge / rsrc_bounds)
    and the min-tree walk decides every row of the pass in ONE batch: groups
    and post-pass state equal to the oracle's, on the serial and the parallel
    host sweeps (NKM_PARALLEL=force)."""
    monkeypatch.setenv("NKM_PARALLEL", par)
    rs = run_passes(config, n, passes, cfg)
    assert rs[0].n_batches == 1, rs[0].n_batches
    assert rs[0].eval_kernel in (6, 7), rs[0].eval_kernel


def test_range_batch_multilevel_sort(monkeypatch):
    """One pool of 40,000 range-source tickets (config 16): 1,024-element
    tiles merged up to runs of 65,536 (6 rsrc_merge launches, the last one
    over a partner run shorter than its own).  The range batch (NKM_RANGE default) must
    form exactly the groups and post-pass state of the list-based replay
    (NKM_RANGE=0), which the oracle pins at the smaller sizes above."""
    def one(rng):
        monkeypatch.setenv("NKM_RANGE", rng)
        ts = synth.TicketSet(16, 40_000)
        mm = capi.Matchmaker(product_lib(), max_intervals=2)
        try:
            ts.insert_into(mm)
            r = mm.process_raw()
            return r, state(mm)
        finally:
            mm.close()
            ts.close()
    got, got_state = one("1")
    want, want_state = one("0")
    assert got.n_batches == 1 and got.eval_kernel in (6, 7), (got.n_batches, got.eval_kernel)
    assert got.eval_kernel == 6 and got.eval_launches == 6, (got.eval_kernel, got.eval_launches)  # merge launches
    assert len(got.groups) > 1000
    assert got.groups == want.groups
    assert got_state == want_state


@pytest.mark.parametrize("mix", ["per_pool", "within_pool"])
def test_range_batch_fields(mix, monkeypatch):
    """Skill-window searches on two numeric fields.  per_pool: each pool (its
    `mode` term) ranges on one field of its own, and the range batch takes the
    pass, one sort per pool.  within_pool: a pool's searches range on both
    fields, so the batch is declined after its sort was issued (mm_range.cpp's
    per-signature field check, which releases the claimed signatures) and the
    other paths decide the pass.  Groups and post-pass state equal to the
    oracle's on both."""
    import random
    monkeypatch.setenv("NKM_PARALLEL", "force")
    rng = random.Random(11)
    n, t0 = 4000, 1_700_000_000_000_000_000
    ts = []
    for i in range(n):
        mode = "m%d" % (i % 2)
        skill, level = rng.randint(0, 3000), rng.randint(0, 100)
        use_level = (i % 2 == 1) if mix == "per_pool" else (i % 3 == 0)
        f, v, w, b = ("level", level, 10, 3) if use_level else ("skill", skill, 200, 50)
        q = ("+properties.mode:%s +properties.%s:>=%d +properties.%s:<=%d properties.%s:>=%d^2 properties.%s:<=%d^2"
             % (mode, f, max(0, v - w), f, v + w, f, max(0, v - b), f, v + b))
        ts.append(capi.Ticket(ticket="t%05d" % i, presences=[capi.Presence("u%d" % i, "s%d" % i, "u%d" % i, "n")],
                              session_id="s%d" % i, party_id="", query=q, min_count=2, max_count=2,
                              string_properties={"mode": mode}, numeric_properties={"skill": float(skill), "level": float(level)},
                              created_at=t0 + 1024 * i, node="node1"))
    gpu, orc = pair(dict(max_intervals=2))
    try:
        gpu.Insert(ts)
        orc.Insert(ts)
        for p in range(2):
            r = gpu.process_raw()
            assert r.groups == orc.Process(), (mix, p)
            assert state(gpu) == state(orc)
            if mix == "per_pool" and p == 0:
                assert r.n_batches == 1 and r.eval_kernel in (6, 7), (r.n_batches, r.eval_kernel)
            if mix == "within_pool" and p == 0:
                assert r.eval_kernel not in (6, 7), r.eval_kernel
    finally:
        gpu.close()
        orc.close()


@pytest.mark.parametrize("partial", ["1", "0"])
def test_c2_partial_parallel_replay(partial, monkeypatch):
    """Truncated variable-score lists under the pool-parallel replay (forced
    at 10k): a pool whose row runs past its list stops there and re-searches,
    the other pools carry on, and the pass restores the reference's group
    order; NKM_PARTIAL=0 replays such batches serially.  (Range batches off.)"""
    monkeypatch.setenv("NKM_RANGE", "0")
    monkeypatch.setenv("NKM_PARALLEL", "force")
    monkeypatch.setenv("NKM_FULLVAR", "0")
    monkeypatch.setenv("NKM_TIER", "0")
    monkeypatch.setenv("NKM_PARTIAL", partial)
    rs = run_passes(2, 10_000, 2, dict(max_intervals=2))
    assert sum(r.n_batches for r in rs) > 2  # truncated lists restarted batches


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("config", [3, 4])
def test_c3_c4_at_6k(config, kernel, monkeypatch):
    """C3 (parties, 5v5) and C4 (64 pools) at 6,000 tickets on every kernel."""
    set_kernel(monkeypatch, kernel)
    run_passes(config, 6000, 2, dict(max_intervals=2))


@pytest.mark.parametrize("kernel", ["mscan", "mhash", "mscan16"])
@pytest.mark.parametrize("config,n,cfg", [(4, 20_000, dict(max_intervals=2)), (3, 20_000, dict(max_intervals=2)),
                                          (1, 10_000, dict(max_intervals=2))])
def test_hashed_mscan(config, n, cfg, kernel, monkeypatch):
    """The hashed mscan (one table probe per candidate, signature-major
    placement over chunks): taken by default here (C4's 64 pool signatures;
    C3's 8 and C1's over a contiguous scan order) and when forced; never
    with "mscan16" (mscan_kernel, or scan_kernel past 16 signatures).  Every
    list must equal the oracle's and the batch must have run on the expected
    kernel (eval_kernel 1 scan, 2 mscan, 4 hashed)."""
    set_kernel(monkeypatch, kernel)
    rs = run_passes(config, n, 2, cfg)
    want = (1 if config == 4 else 2) if kernel == "mscan16" else 4
    assert rs[0].eval_kernel == want


@pytest.mark.parametrize("contig,grid", [("0", "1"), ("1", "1"), ("0", "0"), ("1", "0")])
def test_hashed_mscan_chunk_lengths(contig, grid, monkeypatch):
    """Both chunk shapes of the hashed scan: gathered through the scan order
    and over contiguous slot runs (vector column loads), with ragged first
    and last chunks (the second pass starts past a matched prefix), through
    the key grid or the cuckoo table (NKM_MHGRID).  Lists downloaded
    (NKM_LISTPROOF=0), so every list is placed and read."""
    set_kernel(monkeypatch, "mhash")
    monkeypatch.setenv("NKM_MCONTIG", contig)
    monkeypatch.setenv("NKM_MHGRID", grid)
    monkeypatch.setenv("NKM_LISTPROOF", "0")
    run_passes(4, 9_999, 2, dict(max_intervals=2))
    run_passes(3, 7_777, 2, dict(max_intervals=2))


@pytest.mark.parametrize("mode,count", [("0", "1"), ("1", "1"), ("1", "0"), ("2", "1")])
@pytest.mark.parametrize("config,n,contig", [(3, 20_000, "1"), (4, 20_000, "1"), (3, 7_777, "0"),
                                             (4, 9_999, "0")])
def test_proven_mscan_lists(config, n, contig, mode, count, monkeypatch, capfd):
    """Hashed-scan lists proven equal to their search's batch rows are not
    downloaded (Core::list_proof_mode_): NKM_LISTPROOF=1 (default) skips
    them — with the contiguous scan writing counts only (NKM_MHCOUNT=1,
    default) or the lists as well (0) — 0 downloads every list, 2 downloads
    them and throws if a proven list differs from its rows — over contiguous
    slot runs and through the scan order (NKM_MCONTIG=0).  Groups and state
    equal to the oracle's either way; the profile line reports the proven
    lists."""
    set_kernel(monkeypatch, "mhash")
    monkeypatch.setenv("NKM_MCONTIG", contig)
    monkeypatch.setenv("NKM_LISTPROOF", mode)
    monkeypatch.setenv("NKM_MHCOUNT", count)
    monkeypatch.setenv("NKM_PARALLEL", "force")
    monkeypatch.setenv("NKM_PROFILE", "1")
    rs = run_passes(config, n, 2, dict(max_intervals=2))
    assert rs[0].eval_kernel == 4
    err = capfd.readouterr().err
    got = [tuple(map(int, m)) for m in re.findall(r"\((\d+) of (\d+) proven, \d+ re-run\)", err)]
    assert got, err[-2000:]
    proven = sum(p for p, _ in got)
    assert (proven == 0) if mode == "0" else (proven > 0), got


@pytest.mark.parametrize("config,n", [(3, 9_000), (4, 9_999)])
def test_counts_only_scan_falls_back(config, n, monkeypatch, capfd):
    """Counts-only hashed scans (Core::mhash_count_mode_) expect every list
    proven; with every third ticket inserted inactive (Intervals at
    MaxIntervals: in the index, never a row) the pool lists hold more than
    their rows, the batch re-runs the full scan and downloads them, and the
    speculation pauses.  Groups and state equal to the oracle's."""
    set_kernel(monkeypatch, "mhash")
    monkeypatch.setenv("NKM_MCONTIG", "1")
    monkeypatch.setenv("NKM_PARALLEL", "force")
    monkeypatch.setenv("NKM_PROFILE", "1")
    cfg = dict(max_intervals=2)
    gpu, orc = pair(cfg)
    ts = synth.TicketSet(config, n)
    try:
        for k in range(0, ts.n, 3):
            ts.tickets[k].intervals = 2
        ts.insert_into(gpu)
        ts.insert_into(orc)
        for p in range(2):
            r = gpu.process_raw()
            assert r.groups == orc.Process()
            assert state(gpu) == state(orc)
            if p == 0:
                assert r.eval_kernel == 4
    finally:
        gpu.close()
        orc.close()
        ts.close()
    err = capfd.readouterr().err
    rerun = [int(m) for m in re.findall(r"proven, (\d+) re-run\)", err)]
    assert rerun and rerun[0] >= 1, err[-2000:]


@pytest.mark.parametrize("kernel", KERNELS)
def test_datetime_props_and_date_ranges(kernel, monkeypatch):
    """Config 8: string properties in each layout blugeParseDateTime accepts
    (indexed as raw-UnixNano numeric terms, match_common.go:161-170,221-236)
    mixed with strings none parses (keywords), queried with RFC3339 date-range
    clauses (query_string_parser.go:234-250; ConstantScorer(1))."""
    set_kernel(monkeypatch, kernel)
    run_passes(8, 3000, 3, dict(max_intervals=3))


@pytest.mark.parametrize("config,n,cfg", [(1, 3000, dict(max_intervals=2)), (2, 2500, dict(max_intervals=2)),
                                          (3, 3000, dict(max_intervals=2)), (4, 3000, dict(max_intervals=2)),
                                          (5, 2000, dict(max_intervals=2, rev_precision=True, rev_threshold=0)),
                                          (6, 1500, dict(max_intervals=3)), (7, 1500, dict(max_intervals=2)),
                                          (8, 2000, dict(max_intervals=3)), (10, 1500, dict(max_intervals=2)),
                                          (13, 1500, dict(max_intervals=2, rev_precision=True, rev_threshold=0))])
def test_bulk_insert(config, n, cfg, monkeypatch):
    """Insert on the host workers (mm_insert.cpp), forced at small sizes:
    parties, datetime-typed string properties, numeric and keyword fields,
    regexp / wildcard / fuzzy clauses (their signatures made serially), wide
    queries over builtin fields — passes and state equal to the oracle, and
    the same hit lists as the per-ticket Insert."""
    monkeypatch.setenv("NKM_BULK", "force")
    run_passes(config, n, 2, cfg)
    ts = synth.TicketSet(config, 400)
    monkeypatch.setenv("NKM_BULK", "0")
    ref = capi.Matchmaker(product_lib(), **cfg)
    monkeypatch.setenv("NKM_BULK", "force")
    blk = capi.Matchmaker(product_lib(), **cfg)
    try:
        ts.insert_into(ref)
        ts.insert_into(blk)
        assert state(blk) == state(ref)
        for k in range(0, 400, 17):
            t = ts.ticket_id(k)
            assert blk.debug_hits(t) == ref.debug_hits(t)
    finally:
        ref.close()
        blk.close()
        ts.close()


def test_bulk_insert_falls_back_on_known_ids(monkeypatch):
    """A batch that re-inserts a known id (live, or a dead record a later
    Insert must overwrite) or names one id twice takes the per-ticket path."""
    monkeypatch.setenv("NKM_BULK", "force")
    gpu, orc = pair(dict(max_intervals=3))
    a, b = synth.TicketSet(6, 500), synth.TicketSet(6, 500, first=250)  # b overlaps a by 250 ids
    try:
        for mm in (gpu, orc):
            a.insert_into(mm)
            b.insert_into(mm)
        assert state(gpu) == state(orc)
        assert gpu.Process() == orc.Process()
        for mm in (gpu, orc):
            a.insert_into(mm)  # matched ids come back
        assert state(gpu) == state(orc)
        assert gpu.Process() == orc.Process()
    finally:
        gpu.close()
        orc.close()
        a.close()
        b.close()


@pytest.mark.parametrize("idq", ["party", "ticket"])
def test_bulk_insert_first_id_field_query(idq, monkeypatch):
    """A bulk Insert whose batch holds the first query reading the `party_id`
    or `ticket` field (MapMatchmakerIndex indexes both, match_common.go): the
    batch falls back to the per-ticket path, which fills those columns for its
    own tickets, so searches see every ticket's id terms."""
    monkeypatch.setenv("NKM_BULK", "force")
    n, t0 = 5000, 1_700_000_000_000_000_000
    ts = []
    for i in range(n):
        mode = "m%d" % (i % 3)
        party = "p%d" % (i // 2) if i % 5 == 0 else ""
        q = "+properties.mode:" + mode
        if i % 7 == 0:
            q += (" -party_id:p%d" % ((i // 2 + 1) % (n // 2))) if idq == "party" else \
                 (" -ticket:t%05d properties.mode:%s^2" % ((i + 3) % n, mode))
        ts.append(capi.Ticket(ticket="t%05d" % i, presences=[capi.Presence("u%d" % i, "s%d" % i, "u%d" % i, "n")],
                              session_id="" if party else "s%d" % i, party_id=party, query=q, min_count=2,
                              max_count=3, string_properties={"mode": mode}, created_at=t0 + 1024 * i,
                              node="node1"))  # Extract lists this node's tickets (matchmaker.go:684-720)
    gpu, orc = pair(dict(max_intervals=3))
    try:
        gpu.Insert(ts)
        orc.Insert(ts)
        assert state(gpu) == state(orc)
        for k in range(0, n, 97):
            assert gpu.debug_hits(ts[k].ticket) == orc.debug_hits(ts[k].ticket)
        for _ in range(2):
            assert gpu.Process() == orc.Process()
            assert state(gpu) == state(orc)
    finally:
        gpu.close()
        orc.close()


def test_datetime_hit_lists():
    ts = synth.TicketSet(8, 600)
    gpu, orc = pair(dict(max_intervals=2))
    try:
        ts.insert_into(gpu)
        ts.insert_into(orc)
        for k in range(0, 600, 13):
            t = ts.ticket_id(k)
            hg, ho = gpu.debug_hits(t), orc.debug_hits(t)
            assert [h for h, _ in hg] == [h for h, _ in ho]
            for (_, a), (_, b) in zip(hg, ho):
                assert math.isclose(a, b, rel_tol=1e-6)
    finally:
        gpu.close()
        orc.close()
        ts.close()


@pytest.mark.parametrize("kernel", KERNELS)
def test_wide_queries(kernel, monkeypatch):
    """Config 10: queries over 1-6 distinct keyword / numeric fields with every
    occur: the kernels' preloaded-column evaluation (search/rsmall <= 4 fields,
    scan <= 2) and its per-clause fallback beyond, on every kernel."""
    set_kernel(monkeypatch, kernel)
    run_passes(10, 3000, 3, dict(max_intervals=3))


def test_wide_queries_rev_precision_and_hit_lists():
    """Config 10 with RevPrecision (rsmall / search reverse checks), and its
    hit lists and scores row by row."""
    run_passes(10, 1500, 2, dict(max_intervals=2, rev_precision=True, rev_threshold=0))
    ts = synth.TicketSet(10, 800)
    gpu, orc = pair(dict(max_intervals=2))
    try:
        ts.insert_into(gpu)
        ts.insert_into(orc)
        for k in range(0, 800, 7):
            t = ts.ticket_id(k)
            hg, ho = gpu.debug_hits(t), orc.debug_hits(t)
            assert [h for h, _ in hg] == [h for h, _ in ho]
            for (_, a), (_, b) in zip(hg, ho):
                assert math.isclose(a, b, rel_tol=1e-6)
    finally:
        gpu.close()
        orc.close()
        ts.close()


@pytest.mark.parametrize("config,n,mi", [(5, 800, 2), (6, 600, 3)])
def test_rev_threshold_fired(config, n, mi):
    """RevThreshold (matchmaker.go:244-248): IntervalSec * RevThreshold = 0 s,
    so the timer has fired at the first row and every reverse check is skipped
    (matchmaker_process.go:40-46,139,178) — the pass equals the one without
    RevPrecision."""
    cfg = dict(max_intervals=mi, rev_precision=True, interval_sec=0, rev_threshold=1)
    run_passes(config, n, 2, cfg)
    assert _oracle_passes(config, n, 2, cfg) == _oracle_passes(config, n, 2, dict(max_intervals=mi))


HOST_KERNEL = [("0", "1", "search"), ("force", "1", "scan"), ("force", "1", "mscan"), ("force", "0", "mscan"),
               ("0", "1", "mscan"), ("force", "1", "mhash"), ("force", "1", "mscan16")]


@pytest.mark.parametrize("par,dense,kernel", HOST_KERNEL)
def test_c3_parties_5v5(par, dense, kernel, monkeypatch):
    """NKM_PARALLEL=0: serial host replay/bookkeeping; force: the pool-parallel
    replay and parallel post-pass at any size; NKM_DENSE: dense or generic
    pool walk; NKM_KERNEL: the query-eval kernel."""
    monkeypatch.setenv("NKM_PARALLEL", par)
    monkeypatch.setenv("NKM_DENSE", dense)
    set_kernel(monkeypatch, kernel)
    run_passes(3, 1500, 2, dict(max_intervals=2))


@pytest.mark.parametrize("config,n,passes", [(3, 1500, 2), (4, 1500, 1), (1, 4000, 2)])
@pytest.mark.parametrize("pipe", ["1", "0"])
def test_pipelined_merge(config, n, passes, pipe, monkeypatch):
    """Forced pool-parallel replay with the merge beside the pool walks
    (NKM_PIPE=1: each chunk of rows merged once every walk has passed it) and
    after them (0), against the oracle."""
    monkeypatch.setenv("NKM_PARALLEL", "force")
    monkeypatch.setenv("NKM_PIPE", pipe)
    run_passes(config, n, passes, dict(max_intervals=2))


@pytest.mark.parametrize("par,dense,kernel", HOST_KERNEL)
def test_c4_many_pools(par, dense, kernel, monkeypatch):
    monkeypatch.setenv("NKM_PARALLEL", par)
    monkeypatch.setenv("NKM_DENSE", dense)
    set_kernel(monkeypatch, kernel)
    run_passes(4, 1500, 1, dict(max_intervals=2))


@pytest.mark.parametrize("par,dense,fast", [("0", "1", "1"), ("force", "1", "1"), ("force", "0", "1"),
                                            ("force", "1", "0"), ("0", "1", "0")])
@pytest.mark.parametrize("config,n", [(17, 3000), (17, 12_000), (18, 3000)])
def test_count_multiple_trim_keeps_combo_full(config, n, par, dense, fast, monkeypatch):
    """MaxCount % CountMultiple != 0 (Add accepts it): combos formed at
    l == MaxCount are trimmed and often rejected; Go's stored combo keeps its
    pre-trim length (a slice header is trimmed, matchmaker_process.go:262-271)
    and never takes another hit.  Serial / pool-parallel, dense / generic and
    fast / exact walks (config 17) and the range walk (18) against the oracle;
    the known-answer scenarios CountMultipleTrimRejectedStaysFull-* pin the
    oracle."""
    monkeypatch.setenv("NKM_PARALLEL", par)
    monkeypatch.setenv("NKM_DENSE", dense)
    monkeypatch.setenv("NKM_FAST", fast)
    rs = run_passes(config, n, 3, dict(max_intervals=3))
    if config == 18 and par != "0":  # range batches run on the parallel host paths
        assert rs[0].eval_kernel in (6, 7), rs[0].eval_kernel


@pytest.mark.parametrize("config,n,passes,mi", [(3, 1500, 2, 2), (6, 1000, 3, 3), (4, 1500, 1, 2)])
@pytest.mark.parametrize("par", ["0", "force"])
def test_exact_walk_without_fast_path(config, n, passes, mi, par, monkeypatch):
    """NKM_FAST=0: every row takes the exact loop body even though no two
    tickets share a session (the default takes the fast walks there); both
    serial and pool-parallel replays against the oracle."""
    monkeypatch.setenv("NKM_FAST", "0")
    monkeypatch.setenv("NKM_PARALLEL", par)
    run_passes(config, n, passes, dict(max_intervals=mi))


@pytest.mark.parametrize("par", ["0", "1", "force"])
def test_c5_rev_precision_default_path(par, monkeypatch):
    """NKM_PARALLEL=force: the RevPrecision rows' pool-parallel replay and
    parallel batch assembly at any size (rsmall_kernel's lists either way)."""
    monkeypatch.setenv("NKM_PARALLEL", par)
    run_passes(5, 800, 2, dict(max_intervals=2, rev_precision=True))


@pytest.mark.parametrize("config,n,passes,stride", [(5, 800, 2, 8), (13, 900, 3, 16), (14, 960, 2, 32),
                                                     (11, 640, 2, 64), (6, 600, 3, None)])
@pytest.mark.parametrize("rpack,par", [("1", "0"), ("1", "force"), ("0", "force")])
def test_packed_rev_precision(config, n, passes, stride, rpack, par, monkeypatch):
    """RevPrecision batches whose rows all search short sources run packed
    (rpack_kernel: 64/S rows per wave, fixed-stride lists, narrow pair-matrix
    words, reverse bits) — C5's buckets of 8 (S = 8), config 13's buckets of 12
    with parties, Min < Max and CountMultiple (S = 16), config 14's buckets of
    24 with a required range (S = 32), config 11's buckets of 64 (S = 64) —
    with the serial and the pool-parallel replay, and per row (NKM_RPACK=0:
    rsmall_kernel); config 6's long sources take the per-row path either way."""
    monkeypatch.setenv("NKM_RPACK", rpack)
    monkeypatch.setenv("NKM_PARALLEL", par)
    out = run_passes(config, n, passes, dict(max_intervals=passes, rev_precision=True))
    packed = stride is not None and rpack == "1"
    assert (out[0].eval_kernel == 5) == packed, out[0].eval_kernel


@pytest.mark.parametrize("config,n,passes,rpack", [(5, 800, 2, "1"), (5, 800, 2, "0"), (13, 1800, 3, "1"),
                                                   (14, 3000, 2, "1"), (11, 6400, 2, "1")])
@pytest.mark.parametrize("runs", ["1", "0"])
def test_pool_runs_replay(config, n, passes, rpack, runs, monkeypatch, capfd):
    """Pools that are contiguous runs of the batch (buckets whose tickets
    arrive together, > 64 pools): NKM_RUNS=1 replays each task's row range
    straight into the pass state and copies the tasks' outputs in order
    (replay_runs); 0 keeps per-row records and merge_rows.  Packed and
    per-row (NKM_RPACK=0) RevPrecision lists, against the oracle."""
    monkeypatch.setenv("NKM_PARALLEL", "force")
    monkeypatch.setenv("NKM_RPACK", rpack)
    monkeypatch.setenv("NKM_RUNS", runs)
    monkeypatch.setenv("NKM_PROFILE", "2")
    # RevThreshold 0: no timer (an armed one keeps RevPrecision batches serial)
    out = run_passes(config, n, passes, dict(max_intervals=passes, rev_precision=True, rev_threshold=0))
    assert len(out[0].groups) > 0
    assert ("pool runs:" in capfd.readouterr().err) == (runs == "1")


@pytest.mark.parametrize("pruns", ["1", "0"])
def test_packed_plan_bucket_in_two_runs(pruns, monkeypatch, capfd):
    """Every C5 bucket arriving in two runs (a second set with the same bucket
    names, created after the first): the packed batch's three-sweep plan
    (plan_packed_runs) meets each term again after its run and hands the batch
    to plan_pools' counting sort; NKM_PRUNS=0 goes there directly.  Groups and
    post-pass state equal the oracle's; with contiguous buckets (config 5
    alone) the three-sweep plan is the one taken."""
    monkeypatch.setenv("NKM_PARALLEL", "force")
    monkeypatch.setenv("NKM_PRUNS", pruns)
    monkeypatch.setenv("NKM_PROFILE", "2")
    kw = dict(max_intervals=2, rev_precision=True, rev_threshold=0)
    n = 800
    sets = [synth.TicketSet(5, n), synth.TicketSet(5, n, seed=0x5EED0105, t0=synth.T0 + 1024 * n)]
    gpu = capi.Matchmaker(product_lib(), **kw)
    orc = capi.Matchmaker(harness.oracle_lib(), **kw)
    try:
        for ts in sets:
            ts.insert_into(gpu)
            ts.insert_into(orc)
        for p in range(2):
            g, o = gpu.process_raw(), orc.process_raw()
            assert g.groups == o.groups, f"pass {p}: {len(g.groups)} vs oracle {len(o.groups)} groups"
            assert state(gpu) == state(orc)
            assert p or g.groups
    finally:
        gpu.close()
        orc.close()
        for ts in sets:
            ts.close()
    err = capfd.readouterr().err
    assert "3 sweeps" not in err  # never planned as runs: the buckets come back
    assert ("pool runs:" in err) is False
    out = run_passes(5, n, 1, kw)
    assert len(out[0].groups) > 0
    assert ("3 sweeps" in capfd.readouterr().err) == (pruns == "1")


@pytest.mark.parametrize("direct", ["1", "0"])
@pytest.mark.parametrize("config,n", [(5, 5000), (6, 100), (13, 900)])
def test_custom_candidates_into_result_arena(config, n, direct, monkeypatch):
    """processCustom's device candidates written straight into the result
    arena in pinned chunks (NKM_CDIRECT=1, forced at any size by
    NKM_PARALLEL=force) or through the candidate list and fill_matched (0):
    the override sees the oracle's candidate list either way, and a second
    pass's result while the first is still held takes private copies."""
    monkeypatch.setenv("NKM_PARALLEL", "force")
    monkeypatch.setenv("NKM_CDIRECT", direct)
    monkeypatch.setenv("NKM_DEVENUM", "1")
    seen = {}

    def rec(tag):
        def f(c):
            seen[tag] = [list(x) for x in c]
            return first_disjoint(c)
        return f

    ts = synth.TicketSet(config, n)
    gpu = capi.Matchmaker(product_lib(), override=rec("g"), max_intervals=2, rev_precision=True)
    orc = capi.Matchmaker(harness.oracle_lib(), override=rec("o"), max_intervals=2, rev_precision=True)
    try:
        ts.insert_into(gpu)
        ts.insert_into(orc)
        for _ in range(2):
            seen.clear()
            g, o = gpu.Process(), orc.Process()
            assert seen.get("g") == seen.get("o"), "processCustom candidate lists differ"
            assert g == o
            assert state(gpu) == state(orc)
    finally:
        gpu.close()
        orc.close()
        ts.close()


def first_disjoint(cands):
    """The deterministic override of SURVEY.md 8(d) C5: keep candidates, in
    order, that do not overlap an already kept one."""
    used, out = set(), []
    for g in cands:
        ts = {t for t, _ in g}
        if ts & used:
            continue
        used |= ts
        out.append(g)
    return out


@pytest.mark.parametrize("config,n,devenum", [(5, 400, "1"), (5, 5000, "1"), (5, 5000, "0"), (6, 100, "1"),
                                               (6, 100, "0"), (7, 300, "1")])
def test_c5_override_candidates(config, n, devenum, monkeypatch):
    """processCustom candidates (RevPrecision; C5's buckets of 8, config 6's
    parties, count ranges and CountMultiple — 81k candidates per pass at 100
    tickets — and config 7's multi-term queries) handed to the deterministic
    first-disjoint override of SURVEY 8(d) C5, then committed.  NKM_DEVENUM:
    the subsets enumerated by enum_kernel (1) or on the host (0)."""
    monkeypatch.setenv("NKM_DEVENUM", devenum)
    seen = {}

    def rec(tag):
        def f(c):
            seen[tag] = [list(x) for x in c]
            return first_disjoint(c)
        return f

    ts = synth.TicketSet(config, n)
    gpu = capi.Matchmaker(product_lib(), override=rec("g"), max_intervals=2, rev_precision=True)
    orc = capi.Matchmaker(harness.oracle_lib(), override=rec("o"), max_intervals=2, rev_precision=True)
    try:
        ts.insert_into(gpu)
        ts.insert_into(orc)
        for _ in range(2):
            seen.clear()
            g, o = gpu.Process(), orc.Process()
            assert seen.get("g") == seen.get("o"), "processCustom candidate lists differ"
            assert g == o
            assert state(gpu) == state(orc)
    finally:
        gpu.close()
        orc.close()
        ts.close()


@pytest.mark.parametrize("par,dense,kernel", HOST_KERNEL)
def test_mixed_parties_ranges_minmax(par, dense, kernel, monkeypatch):
    monkeypatch.setenv("NKM_PARALLEL", par)
    monkeypatch.setenv("NKM_DENSE", dense)
    set_kernel(monkeypatch, kernel)
    run_passes(6, 1000, 3, dict(max_intervals=3))


@pytest.mark.parametrize("page,par", [("1", "1"), ("0", "1"), ("1", "force")])
def test_mixed_rev_precision(page, par, monkeypatch):
    monkeypatch.setenv("NKM_PAGE", page)
    monkeypatch.setenv("NKM_PARALLEL", par)
    run_passes(6, 600, 3, dict(max_intervals=3, rev_precision=True))


def test_paused_pass_bumps_intervals():
    ts = synth.TicketSet(6, 200)
    gpu, orc = pair(dict(max_intervals=3))
    try:
        ts.insert_into(gpu)
        ts.insert_into(orc)
        gpu.Pause()
        orc.Pause()
        assert gpu.Process() == orc.Process() == []
        assert state(gpu) == state(orc)
        gpu.Resume()
        orc.Resume()
        assert gpu.Process() == orc.Process()
        assert state(gpu) == state(orc)
    finally:
        gpu.close()
        orc.close()
        ts.close()


def test_interleaved_mutations():
    """Insert / remove / add between passes (store maintenance + compaction)."""
    gpu, orc = pair(dict(max_intervals=2, max_tickets=3))
    sets = []
    try:
        for rnd in range(4):
            ts = synth.TicketSet(6, 300, first=rnd * 300)
            sets.append(ts)
            ts.insert_into(gpu)
            ts.insert_into(orc)
            # remove a few tickets by id
            victims = [ts.ticket_id(k) for k in range(0, 300, 37)]
            gpu.Remove(victims)
            orc.Remove(victims)
            for k in range(1, 300, 53):
                t = ts.tickets[k]
                if t.n_presences == 1:
                    sid = t.presences[0].session_id.decode()
                    gpu.RemoveSessionAll(sid)
                    orc.RemoveSessionAll(sid)
            assert gpu.Process() == orc.Process()
            assert state(gpu) == state(orc)
            assert gpu.ticket_count() == orc.ticket_count()
    finally:
        gpu.close()
        orc.close()
        for s in sets:
            s.close()


def test_drained_store_compacts_and_refills():
    """Every ticket removed, then an Insert: the compaction takes the drained
    store's shortcut (columns emptied, the cold records' buffer kept) and the
    refilled store passes like the oracle's — twice, so the second drain
    reuses the first refill's buffers."""
    gpu, orc = pair(dict(max_intervals=2))
    big = synth.TicketSet(3, 70_000)
    try:
        for rnd in range(2):
            small = synth.TicketSet(6, 500, first=100_000 * (rnd + 1))
            big.insert_into(gpu)
            big.insert_into(orc)
            ids = [t.ticket for t in gpu.Extract()]
            gpu.Remove(ids)
            orc.Remove(ids)
            assert gpu.ticket_count() == orc.ticket_count() == 0
            small.insert_into(gpu)  # compacts: 70,000+ slots, none live
            small.insert_into(orc)
            assert state(gpu) == state(orc)
            assert gpu.Process() == orc.Process()
            assert state(gpu) == state(orc)
            rest = [t.ticket for t in gpu.Extract()]
            gpu.Remove(rest)
            orc.Remove(rest)
            small.close()
    finally:
        gpu.close()
        orc.close()
        big.close()


def test_store_compaction_extract_and_replace():
    """Store maintenance at a size that compacts (>= 65,536 slots, over half
    dead): bulk Insert, mass Remove, the compaction on the next Insert, ids
    re-inserted within and across batches (replace), RemoveAll by node, and
    the full Extract / pass results against the oracle after each step."""
    gpu, orc = pair(dict(max_intervals=3, max_tickets=3))
    big = synth.TicketSet(3, 70_000)
    small = synth.TicketSet(6, 400, first=70_000)
    try:
        big.insert_into(gpu)
        big.insert_into(orc)
        assert gpu.ticket_count() == orc.ticket_count() == 70_000
        keep = set(range(0, 70_000, 151))
        victims = [big.ticket_id(k) for k in range(70_000) if k not in keep]
        gpu.Remove(victims)
        orc.Remove(victims)
        small.insert_into(gpu)  # compacts: 70,400 slots, ~860 live
        small.insert_into(orc)
        assert state(gpu) == state(orc)
        assert gpu.Process() == orc.Process()
        assert state(gpu) == state(orc)
        small.insert_into(gpu)  # every id again: replaced in place of the old slots
        small.insert_into(orc)
        assert gpu.ticket_count() == orc.ticket_count()
        assert state(gpu) == state(orc)
        assert gpu.Process() == orc.Process()
        assert state(gpu) == state(orc)
        nodes = sorted({t.node for t in gpu.Extract()})
        if nodes:
            gpu.RemoveAll(nodes[0])
            orc.RemoveAll(nodes[0])
        assert state(gpu) == state(orc)
        assert gpu.Process() == orc.Process()
    finally:
        gpu.close()
        orc.close()
        big.close()
        small.close()


@pytest.mark.parametrize("config", [1, 2, 3, 5, 6])
def test_hit_lists_and_scores(config):
    """Per-ticket search results: same hits, same order, scores within 1e-6."""
    ts = synth.TicketSet(config, 500)
    gpu, orc = pair(dict(max_intervals=2))
    try:
        ts.insert_into(gpu)
        ts.insert_into(orc)
        for k in range(0, 500, 41):
            t = ts.ticket_id(k)
            hg, ho = gpu.debug_hits(t), orc.debug_hits(t)
            assert [h for h, _ in hg] == [h for h, _ in ho]
            for (_, a), (_, b) in zip(hg, ho):
                assert math.isclose(a, b, rel_tol=1e-6)
    finally:
        gpu.close()
        orc.close()
        ts.close()


@pytest.mark.parametrize("n", [20_000])
def test_large_pool_properties(n):
    """Size-independent properties at a size the oracle cannot check directly:
    every group has MaxCount presences, a multiple of CountMultiple, shares
    the pool key, never repeats a ticket, and every matched ticket left the pool."""
    ts = synth.TicketSet(3, n)
    gpu = capi.Matchmaker(product_lib(), max_intervals=2)
    props = {}
    for k in range(n):
        t = ts.tickets[k]
        props[t.ticket.decode()] = tuple(t.str_props[j].value for j in range(t.n_str_props))
    try:
        ts.insert_into(gpu)
        groups = gpu.Process()
        seen = set()
        for g in groups:
            assert len(g) == 10
            tickets = {t for t, _ in g}
            assert len({props[t] for t in tickets}) == 1
            assert not (tickets & seen)
            seen |= tickets
        assert gpu.ticket_count() == n - len(seen)
        assert len(seen) > 0.9 * n
    finally:
        gpu.close()
        ts.close()


def _product_passes(config, n, passes, par, monkeypatch, dense="1", kernel="auto", fast="1"):
    monkeypatch.setenv("NKM_PARALLEL", par)
    monkeypatch.setenv("NKM_DENSE", dense)
    set_kernel(monkeypatch, kernel)
    monkeypatch.setenv("NKM_FAST", fast)
    ts = synth.TicketSet(config, n)
    mm = capi.Matchmaker(product_lib(), max_intervals=2)
    try:
        ts.insert_into(mm)
        out = []
        for _ in range(passes):
            out.append(mm.Process())
            out.append(state(mm))
        return out
    finally:
        mm.close()
        ts.close()


@pytest.mark.parametrize("config,n", [(3, 300_000), (4, 200_000)])
def test_parallel_host_paths_equal_serial(config, n, monkeypatch):
    """At sizes past the oracle's reach, the pool-parallel replay and the
    parallel post-pass, with the fast (exclusive-session) walks, give exactly
    the serial exact path's groups and state (the serial path is the one
    checked against the oracle above); mscan_kernel's look-back runs over ~300
    chunks here."""
    ser = _product_passes(config, n, 2, "0", monkeypatch, kernel="scan", fast="0")
    par = _product_passes(config, n, 2, "1", monkeypatch)
    assert par == ser
    gen = _product_passes(config, n, 2, "1", monkeypatch, dense="0", kernel="mscan")
    assert gen == ser
    exact = _product_passes(config, n, 2, "1", monkeypatch, fast="0")
    assert exact == ser
    monkeypatch.setenv("NKM_PIPE", "0")  # the merge after all pool walks instead of beside them
    nopipe = _product_passes(config, n, 2, "1", monkeypatch)
    monkeypatch.delenv("NKM_PIPE")
    assert nopipe == ser


# ---- regexp / wildcard / fuzzy clauses (OP_TERMSET) ----

@pytest.mark.parametrize("case", KA["search_cases"], ids=[c["name"] for c in KA["search_cases"]])
def test_regexp_search_cases_gpu(case):
    """TestMatchmakerPropertyRegexSubmatch{,Multiple} through the device search."""
    hit, hits = harness.search_case_hit(product_lib(), case, KA["T0"])
    assert hit == case["hit"], (case["name"], hits)
    assert hits == harness.search_case_hit(harness.oracle_lib(), case, KA["T0"])[1]


@pytest.mark.parametrize("kernel,page,fullvar", [("search", "1", "1"), ("scan", "1", "1"), ("mscan", "1", "1"),
                                                 ("search", "0", "1"), ("search", "1", "0")])
def test_multi_term_passes(kernel, page, fullvar, monkeypatch):
    """Config 7: blocked-list regexps, alternations, wildcards, fuzzy (variable
    scores), a pattern that fails every search; every query-eval kernel;
    truncated lists paged by any row (NKM_PAGE=1) or by batch restarts."""
    set_kernel(monkeypatch, kernel)
    monkeypatch.setenv("NKM_PAGE", page)
    monkeypatch.setenv("NKM_FULLVAR", fullvar)
    rs = run_passes(7, 1200, 3, dict(max_intervals=3))
    full = sum(r.full_lists for r in rs)
    if fullvar == "0":
        assert full == 0
    elif kernel == "search":
        assert full > 0  # the full-list branch ran


def test_multi_term_rev_precision():
    run_passes(7, 600, 2, dict(max_intervals=2, rev_precision=True))


def test_multi_term_hit_lists():
    ts = synth.TicketSet(7, 600)
    gpu, orc = pair(dict(max_intervals=2))
    try:
        ts.insert_into(gpu)
        ts.insert_into(orc)
        for k in range(0, 600, 7):
            t = ts.ticket_id(k)
            hg, ho = gpu.debug_hits(t), orc.debug_hits(t)
            assert [h for h, _ in hg] == [h for h, _ in ho]
            for (_, a), (_, b) in zip(hg, ho):
                assert math.isclose(a, b, rel_tol=1e-6)
    finally:
        gpu.close()
        orc.close()
        ts.close()


def test_multi_term_sets_grow_between_passes():
    """Terms interned after a pattern was first evaluated join its set."""
    gpu, orc = pair(dict(max_intervals=3))
    sets = []
    try:
        for rnd in range(3):
            ts = synth.TicketSet(7, 250, first=rnd * 250)
            sets.append(ts)
            ts.insert_into(gpu)
            ts.insert_into(orc)
            assert gpu.Process() == orc.Process()
            assert state(gpu) == state(orc)
    finally:
        gpu.close()
        orc.close()
        for s in sets:
            s.close()


def _custom_many_hits(lib, n_tickets):
    """n_tickets tickets with query "*", Min=2 Max=3: every row has
    n_tickets-1 filtered hits (> 40, < 63), so combineIndexes' ascending mask
    loop (matchmaker_process.go:578-612) emits every 2-subset (hitCount 3;
    1-subsets reach hitCount 2 < MaxCount and are rejected, :496)."""
    seen = []
    mm = capi.Matchmaker(lib, override=lambda c: (seen.append([list(g) for g in c]), [])[1], max_intervals=5)
    try:
        for i in range(n_tickets):
            mm.Add([capi.Presence(f"u{i}", f"s{i}", f"u{i}", "n")], f"s{i}", "", "*", 2, 3, 1, {"k": "v"}, {},
                   ticket=f"t{i:03d}", created_at=synth.T0 + 1024 * i)
        mm.Process()
        return seen[0] if seen else []
    finally:
        mm.close()


@pytest.mark.parametrize("devenum", ["1", "0"])
def test_custom_zero_candidates_at_63_hits(devenum, monkeypatch):
    """Rows with 63 / 64 filtered hits hand over no candidate (Go's `1 <<
    length` overflow, matchmaker_process.go:588) while rows of 62 and 4 hits
    in the same pass hand over theirs; the device (enum_kernel) and host
    enumerations both equal the oracle's list."""
    from math import comb
    monkeypatch.setenv("NKM_DEVENUM", devenum)
    got, pool_of = harness.custom_pool_candidates(product_lib())
    want, _ = harness.custom_pool_candidates(harness.oracle_lib())
    assert len(got) == 63 * comb(62, 2) + 5 * comb(4, 2)
    assert not any(pool_of[g[-1][0]] in ("a", "b") for g in got)
    assert got == want


@pytest.mark.parametrize("devenum", ["1", "0"])
def test_custom_rows_past_40_hits(devenum, monkeypatch):
    monkeypatch.setenv("NKM_DEVENUM", devenum)
    n = 51
    cands = _custom_many_hits(product_lib(), n)
    assert len(cands) == n * (n - 1) * (n - 2) // 2
    assert cands == _custom_many_hits(harness.oracle_lib(), n)
