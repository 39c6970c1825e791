"""The bench's override step (tools/synth.cpp synth_override_first_disjoint +
mm_process_commit, nakama_amd/synth.override_commit) against the same override
written in Python through Matchmaker.Process — on the oracle library (CPU)."""
import harness
from nakama_amd import capi, synth


def first_disjoint(groups):
    taken, kept = set(), []
    for g in groups:
        ts = {t for t, _ in g}
        if ts & taken:
            continue
        taken |= ts
        kept.append(g)
    return kept


def test_native_override_equals_python_override():
    lib = harness.oracle_lib()
    ts = synth.TicketSet(5, 400)
    a = capi.Matchmaker(lib, max_intervals=2, rev_precision=True, rev_threshold=0, override=first_disjoint)
    b = capi.Matchmaker(lib, max_intervals=2, rev_precision=True, rev_threshold=0, override=lambda g: g)
    try:
        ts.insert_into(a)
        ts.insert_into(b)
        want = a.Process()
        out = b.process_call()
        assert out.is_candidates
        res = synth.override_commit(b, out)
        try:
            got = capi.Matchmaker._groups(res)
        finally:
            b.lib.mm_free_matched(b.h, capi.C.byref(res))
        assert got == want and len(got) > 0
        assert b.ticket_count() == a.ticket_count()
    finally:
        a.close()
        b.close()
        ts.close()
