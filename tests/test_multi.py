"""One handle over several sub-handles (mm_create_multi, include/nakama_cluster.h).

The reference runs ONE matchmaker per process (main.go:160) behind
server.Matchmaker (server/matchmaker.go:169-183); the multi handle keeps that
contract over one sub-handle per device, driven from host threads in C++.
The CPU tests run the product's front over the CPU oracle's handles (the
front is library code; only the sub-handles' library changes) and compare
every observable with ONE oracle handle fed the same calls: groups and
their order, processCustom candidate lists, the override's commit (including
an override that reorders and overlaps groups: the post-pass re-check and
its swap-remove), the post-pass state, MaxTickets across pools and every
Remove* routed or broadcast.  The GPU tests run the same comparisons with
HIP sub-handles (two on device 0), in both modes.
"""
import ctypes as C

import pytest

import harness
from nakama_amd import capi, synth

POOL_FIELDS = {1: ["properties.mode", "properties.region"], 2: ["properties.region"], 15: ["properties.region"],
               3: ["properties.mode", "properties.region"],
               4: ["properties.mode", "properties.region"], 5: ["properties.bucket"], 12: ["properties.mode"]}


def product_lib():
    return capi.load_library(harness.PRODUCT_SO)


def multi(n, config, sub_lib, mode=capi.MM_MULTI_POOLS, transport=capi.MM_MULTI_AUTO, devices=None, **kw):
    return capi.Matchmaker(product_lib(), multi=dict(devices=devices or [0] * n, mode=mode,
                                                     pool_fields=POOL_FIELDS.get(config, []), transport=transport,
                                                     sub_lib=sub_lib), **kw)


def state(mm):
    return mm.Extract(), mm.active_count(), mm.ticket_count()


def reversing_overlapping(cands):
    """An override that returns the candidates in reverse order, overlapping:
    the post-pass re-check drops every group that lost a ticket to an earlier
    one, with the reference's swap-remove (matchmaker.go:326-343)."""
    return list(reversed(cands))[: max(1, len(cands) // 3)]


def _compare(config, n, passes, sub_lib, n_subs=2, override=None, **kw):
    ts = synth.TicketSet(config, n)
    one = capi.Matchmaker(harness.oracle_lib(), override=override, **kw)
    mm = multi(n_subs, config, sub_lib, override=override, **kw)
    try:
        ts.insert_into(one)
        ts.insert_into(mm)
        assert state(mm) == state(one)
        for p in range(passes):
            seen = {}
            if override is not None:
                one.override = lambda c: (seen.__setitem__("one", c), override(c))[1]
                mm.override = lambda c: (seen.__setitem__("mm", c), override(c))[1]
            g1, gm = one.Process(), mm.Process()
            assert gm == g1, f"pass {p}: groups differ ({len(gm)} vs {len(g1)})"
            assert seen.get("mm") == seen.get("one"), f"pass {p}: candidate lists differ"
            assert state(mm) == state(one)
        return mm.lib.mm_multi_info(mm.h, -1)
    finally:
        mm.close()
        one.close()
        ts.close()


# ---- CPU: the front over oracle sub-handles ----

@pytest.mark.parametrize("config,n,subs", [(3, 3000, 2), (3, 3000, 3), (4, 3000, 4), (12, 600, 2), (12, 900, 3)])
def test_multi_pools_default_pass_equals_one_handle(config, n, subs):
    """processDefault over pools placed whole on sub-handles, merged by the
    searching ticket (CreatedAt, Ticket): config 3 (parties, 5v5), config 4
    (64 pools), config 12 (config 6 pinned to its mode:
    parties, Min<Max, CountMultiple)."""
    assert _compare(config, n, 3, harness.oracle_lib(), n_subs=subs, max_intervals=3) == subs


@pytest.mark.parametrize("config,n,subs", [(3, 3000, 3), (4, 3000, 4), (12, 900, 3)])
def test_multi_pools_parallel_merge(config, n, subs, monkeypatch):
    """The key-range parallel merge of the sub-handles' lists (forced at any
    size): the same groups, in the same order, as one handle."""
    monkeypatch.setenv("NKM_PARALLEL", "force")
    assert _compare(config, n, 2, harness.oracle_lib(), n_subs=subs, max_intervals=3) == subs


def test_multi_pools_parallel_merge_ties():
    """Groups of different sub-handles whose searching tickets share a
    CreatedAt are ordered by ticket id (the pinned active order); the
    parallel merge keeps every tie inside one key range."""
    def run(m):
        for k in range(240):
            mode = f"m{k % 3}"
            for j in range(2):
                _add(m, f"t{k:03d}-{j}", [f"s{k}-{j}"], query=f"+properties.mode:{mode}", props={"mode": mode},
                     created=k // 6)
        return m.Process()
    import os
    os.environ["NKM_PARALLEL"] = "force"
    try:
        _both(run)
    finally:
        del os.environ["NKM_PARALLEL"]


def test_multi_pools_rev_precision():
    _compare(5, 1200, 2, harness.oracle_lib(), n_subs=3, max_intervals=2, rev_precision=True, rev_threshold=0)


@pytest.mark.parametrize("override", ["first-disjoint", "reverse-overlap"])
def test_multi_pools_override_hand_off(override):
    """processCustom candidates merged across sub-handles in the reference's
    order; the override's choice committed with the global re-check."""
    from test_gpu_parity import first_disjoint
    fn = first_disjoint if override == "first-disjoint" else reversing_overlapping
    _compare(5, 800, 2, harness.oracle_lib(), n_subs=3, override=fn, max_intervals=2, rev_precision=True,
             rev_threshold=0)


def test_multi_pools_override_groups_spanning_pools():
    """An override may return any group: one that mixes pools is committed
    in parts on the sub-handles and reassembled in entry order."""
    def mix(cands):
        out = []
        for a, b in zip(cands[::2], cands[1::2]):
            out.append(a + b)
        return out
    _compare(12, 60, 2, harness.oracle_lib(), n_subs=2, override=mix, max_intervals=3)


def _add(mm, t, sids, party="", query=None, props=None, created=0, count=None):
    pres = [capi.Presence(f"u-{s}", s, f"u-{s}", "n") for s in sids]
    return mm.Add(pres, sids[0] if not party else "", party, query, 2, 2, 1, props, {}, ticket=t,
                  created_at=synth.T0 + 1024 * created)


def _both(fn):
    one = capi.Matchmaker(harness.oracle_lib(), max_tickets=3, max_intervals=3)
    mm = capi.Matchmaker(product_lib(), max_tickets=3, max_intervals=3,
                         multi=dict(devices=[0, 0, 0], pool_fields=["properties.mode"], sub_lib=harness.oracle_lib()))
    try:
        r1, rm = fn(one), fn(mm)
        assert rm == r1
        assert state(mm) == state(one)
        return mm
    finally:
        mm.close()
        one.close()


def _errs(mm, calls):
    out = []
    for c in calls:
        try:
            c(mm)
            out.append(None)
        except capi.MatchmakerError as e:
            out.append(type(e).__name__)
    return out


def test_multi_max_tickets_across_pools():
    """MaxTickets per session and per party (matchmaker.go:508-521) counts
    the tickets of every sub-handle: one session's tickets in three pools."""
    modes = ["m0", "m1", "m2", "m3"]
    calls = [lambda m, k=k: _add(m, f"t{k}", ["s1"], query=f"+properties.mode:{modes[k]}",
                                 props={"mode": modes[k]}, created=k) for k in range(4)]
    calls += [lambda m, k=k: _add(m, f"p{k}", ["ps1", "ps2"], party="party1", query=f"+properties.mode:{modes[k]}",
                                  props={"mode": modes[k]}, created=10 + k) for k in range(4)]
    # after one is removed, the session may add again
    calls.append(lambda m: m.RemoveSession("s1", "t1"))
    calls.append(lambda m: _add(m, "t9", ["s1"], query="+properties.mode:m3", props={"mode": "m3"}, created=20))
    calls.append(lambda m: m.RemoveParty("party1", "p0"))
    calls.append(lambda m: _add(m, "p9", ["ps1", "ps2"], party="party1", query="+properties.mode:m3",
                                props={"mode": "m3"}, created=21))
    r = _both(lambda m: _errs(m, calls))
    assert r is not None


def test_multi_removals_routed_and_broadcast():
    """Remove* reach the sub-handle holding the ticket (RemoveSession /
    RemoveParty / Remove) or every sub-handle (RemoveSessionAll /
    RemovePartyAll / RemoveAll); a removed ticket is never matched."""
    def run(m):
        ts = synth.TicketSet(12, 400)
        try:
            ts.insert_into(m)
            ids = [ts.ticket_id(k) for k in range(0, 400, 9)]
            m.Remove(ids)
            out = []
            for k in range(1, 400, 23):
                t = ts.tickets[k]
                if t.n_presences == 1:
                    out += _errs(m, [lambda mm, t=t: mm.RemoveSession(t.presences[0].session_id.decode(),
                                                                      t.ticket.decode())])
                    out += _errs(m, [lambda mm, t=t: mm.RemoveSession("nope", t.ticket.decode())])
                else:
                    out += _errs(m, [lambda mm, t=t: mm.RemovePartyAll(t.party_id.decode())])
            for k in range(2, 400, 31):
                t = ts.tickets[k]
                m.RemoveSessionAll(t.presences[0].session_id.decode())
            out.append(m.Process())
            m.RemoveAll("node1")
            out.append(m.ticket_count())
            return out
        finally:
            ts.close()
    _both(run)


def test_multi_drain_removed():
    """mm_drain_removed of the multi handle: tickets that left any sub-handle."""
    def run(m):
        ts = synth.TicketSet(12, 300)
        try:
            m.drain_removed()
            ts.insert_into(m)
            m.Remove([ts.ticket_id(k) for k in range(0, 300, 7)])
            a = sorted(m.drain_removed())
            groups = m.Process()
            b = sorted(m.drain_removed())
            return a, b, sorted({t for g in groups for t, _ in g})
        finally:
            ts.close()
    _both(run)


def test_multi_lookups_across_sub_handles():
    """mm_session_ticket_count / mm_party_ticket_count / mm_find_tickets of the
    multi handle (ABI 4) answer for every sub-handle: a session's and a
    party's tickets in three pools, found wherever they live."""
    def run(m):
        modes = ["m0", "m1", "m2"]
        for k in range(3):
            _add(m, f"t{k}", ["s1"], query=f"+properties.mode:{modes[k]}", props={"mode": modes[k]}, created=k)
            _add(m, f"p{k}", ["ps1", "ps2"], party="party1", query=f"+properties.mode:{modes[k]}",
                 props={"mode": modes[k]}, created=10 + k)
        out = [m.session_ticket_count("s1"), m.session_ticket_count("ps2"), m.party_ticket_count("party1"),
               m.session_ticket_count("nobody"), m.party_ticket_count(""),
               m.find_tickets(["t0", "t2", "p1", "zz", "t1"])]
        m.RemoveSession("s1", "t2")
        out += [m.session_ticket_count("s1"), m.find_tickets(["t2", "t0"])]
        return out
    _both(run)


def test_multi_unroutable_ticket_refused():
    """MM_MULTI_POOLS serves tickets whose query pins every pool field to the
    ticket's own value; any other is refused (ErrMatchmakerUnsupportedQuery),
    an invalid query is ErrMatchmakerQueryInvalid as for one handle."""
    mm = capi.Matchmaker(product_lib(), multi=dict(devices=[0, 0], pool_fields=["properties.mode"],
                                                   sub_lib=harness.oracle_lib()))
    try:
        with pytest.raises(capi.ErrMatchmakerUnsupportedQuery):
            _add(mm, "a", ["s1"], query="+properties.mode:x", props={"mode": "y"})
        with pytest.raises(capi.ErrMatchmakerUnsupportedQuery):
            _add(mm, "b", ["s2"], query="*", props={"mode": "y"})
        with pytest.raises(capi.ErrMatchmakerQueryInvalid):
            _add(mm, "c", ["s3"], query="+properties.mode:", props={"mode": "y"})
        _add(mm, "d", ["s4"], query="+properties.mode:y", props={"mode": "y"})
        assert mm.ticket_count() == 1
    finally:
        mm.close()


def test_multi_rows_mode_needs_own_library():
    with pytest.raises(capi.ErrDevice):
        capi.Matchmaker(product_lib(), multi=dict(devices=[0, 0], mode=capi.MM_MULTI_ROWS,
                                                  sub_lib=harness.oracle_lib()))


# ---- GPU: HIP sub-handles ----

@pytest.mark.gpu
@pytest.mark.parametrize("config,n,kw", [(3, 6000, dict(max_intervals=2)), (4, 6000, dict(max_intervals=2)),
                                         (12, 1000, dict(max_intervals=3)),
                                         (5, 2000, dict(max_intervals=2, rev_precision=True, rev_threshold=0)),
                                         (2, 6000, dict(max_intervals=2)), (15, 3000, dict(max_intervals=3))])
def test_gpu_multi_pools_equal_one_oracle(config, n, kw):
    """Two HIP sub-handles on device 0, pools placed whole, vs one oracle pass
    (configs 2 and 15: each sub-handle's pass a range batch)."""
    _compare(config, n, 2, None, n_subs=2, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("override", ["first-disjoint", "reverse-overlap"])
def test_gpu_multi_pools_override(override):
    from test_gpu_parity import first_disjoint
    fn = first_disjoint if override == "first-disjoint" else reversing_overlapping
    _compare(5, 3000, 2, None, n_subs=2, override=fn, max_intervals=2, rev_precision=True, rev_threshold=0)


@pytest.mark.gpu
@pytest.mark.parametrize("config,n,kw", [(9, 4000, dict(max_intervals=2)), (2, 6000, dict(max_intervals=2)),
                                         (6, 1000, dict(max_intervals=3)),
                                         (6, 600, dict(max_intervals=3, rev_precision=True, rev_threshold=0))])
def test_gpu_multi_rows_host_exchange(config, n, kw):
    """MM_MULTI_ROWS: every sub-handle holds every ticket, the batch searches
    are split between the two sub-handles (device 0 twice: the host-memory
    exchange) and both replay the same lists; config 9's skill windows cross
    the region pools."""
    ts = synth.TicketSet(config, n)
    one = capi.Matchmaker(harness.oracle_lib(), **kw)
    mm = multi(2, config, None, mode=capi.MM_MULTI_ROWS, transport=capi.MM_MULTI_HOST, **kw)
    try:
        ts.insert_into(one)
        ts.insert_into(mm)
        for _ in range(2):
            assert mm.Process() == one.Process()
            assert state(mm) == state(one)
        assert mm.lib.mm_multi_info(mm.h, 1) == one.ticket_count()  # the replica agrees
    finally:
        mm.close()
        one.close()
        ts.close()


@pytest.mark.gpu
@pytest.mark.parametrize("config,n", [(4, 12_000), (3, 9_000)])
def test_gpu_multi_rows_hashed_scan(config, n, monkeypatch):
    """MM_MULTI_ROWS on C4's shape (64 mode x region pools) and C3's: the
    pool signatures run on the hashed scan split by candidate chunks between
    the two sub-handles (the blocks' chunk outputs exchanged through host
    memory, every sub-handle placing every list), equal to one oracle pass;
    eval_kernel 4 = mscan_hash_kernel."""
    monkeypatch.setenv("NKM_KERNEL", "mscan")
    kw = dict(max_intervals=2)
    ts = synth.TicketSet(config, n)
    one = capi.Matchmaker(harness.oracle_lib(), **kw)
    mm = multi(2, config, None, mode=capi.MM_MULTI_ROWS, transport=capi.MM_MULTI_HOST, **kw)
    try:
        ts.insert_into(one)
        ts.insert_into(mm)
        for p in range(2):
            r = mm.process_raw()
            assert r.groups == one.Process(), f"pass {p}"
            assert state(mm) == state(one)
            if p == 0:
                assert r.eval_kernel == 4
    finally:
        mm.close()
        one.close()
        ts.close()


@pytest.mark.gpu
def test_gpu_multi_rows_mutations_during_pass_wait_for_it():
    """MM_MULTI_ROWS: a mutator called while a pass runs waits for the pass
    to end and then reaches every replica, so the replicas never diverge (a
    mutation seen by one replica's pass and not another's would split their
    searches).  Equal to the oracle running the same mutations after its pass."""
    import threading

    from test_concurrency import _mutations, _state

    def run(mm, concurrent):
        base = synth.TicketSet(6, 400)
        extra = synth.TicketSet(6, 300, first=400)
        try:
            base.insert_into(mm)
            mm.drain_removed()
            statuses, err = [], []

            def mutate():
                try:
                    _mutations(mm, base, extra, statuses)
                except Exception as e:  # surfaced below
                    err.append(e)
            th = threading.Thread(target=mutate)
            if concurrent:
                mm.set_pass_hook(th.start)  # the mutations start inside sub-handle 0's pass
                groups = mm.Process()
                th.join(120)
                mm.set_pass_hook(None)
            else:
                groups = mm.Process()
                th.start()
                th.join(120)
            assert not th.is_alive() and not err, err
            out = [groups, statuses, _state(mm), sorted(mm.drain_removed()), mm.Process(), _state(mm),
                   sorted(mm.drain_removed())]
            if concurrent:
                assert mm.lib.mm_multi_info(mm.h, 1) == mm.ticket_count()  # the replicas agree
            return out
        finally:
            mm.close()
            base.close()
            extra.close()

    got = run(multi(2, 6, None, mode=capi.MM_MULTI_ROWS, transport=capi.MM_MULTI_HOST, max_tickets=3, max_intervals=3),
              True)
    want = run(capi.Matchmaker(harness.oracle_lib(), max_tickets=3, max_intervals=3), False)
    names = ["groups", "statuses", "state", "removed", "next groups", "next state", "next removed"]
    for name, a, b in zip(names, got, want):
        assert a == b, name
