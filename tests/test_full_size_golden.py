"""The product's full-size passes against the oracle's (needs a gfx950 GPU).

tests/golden/full_<name>.json holds, for one Process() over the bench-sized
synthetic set of a BASELINE config (C2 100k, C3 1M, C4 4M, C5 1M with
RevPrecision, C5 1M + MatchmakerOverride), the SHA-256 of the oracle's ordered
groups (and processCustom candidate list) and of its post-pass state,
produced offline by tools/make_full_golden.py (per-pool / per-bucket-chunk
oracle runs recombined exactly; see its docstring).  Here the HIP library runs
the same pass on the whole set through the C ABI — crossing every size
threshold the small parity tests do not reach (batch and hit budgets, mscan's
thousands of chunks, the pipelined merge over 125k-row pools) — and its
digests must be equal: bit-exact groups, entry order, group order, candidate
order, and the remaining tickets' intervals.
"""
import ctypes as C
import json
import os

import pytest

import harness
from nakama_amd import capi, synth

pytestmark = pytest.mark.gpu

NAMES = ["c2", "c3", "c4", "c5", "c5o"]


def _golden(name):
    path = os.path.join(harness.GOLDEN, f"full_{name}.json")
    # every BASELINE config's fixture is required: a missing one fails (a skip
    # would let a green run hide an unpinned config)
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: generate it with tools/make_full_golden.py {name}")
    with open(path) as f:
        return json.load(f)


def _product_pass(g, multi=None):
    import nakama_amd
    lib = nakama_amd.load_library()
    kw = dict(g["matchmaker"])
    ts = synth.TicketSet(g["config"], g["tickets"])
    mm = capi.Matchmaker(lib, override=(lambda c: c) if g["override"] else None, multi=multi, **kw)
    got = {}
    try:
        ts.insert_into(mm)
        out = mm.process_call()
        if g["override"]:
            assert out.is_candidates
            cd = synth.Digest()
            got["candidates"] = out.n_groups
            got["candidate_entries"] = cd.groups_raw(out)
            got["candidates_sha256"] = cd.hexdigest()
            out = synth.override_commit(mm, out)
        try:
            gd = synth.Digest()
            got["groups"] = out.n_groups
            got["entries"] = gd.groups_raw(out)
            got["groups_sha256"] = gd.hexdigest()
            got["matched_tickets"] = mm.summary_counts(out)[1]
            got["eval_kernel"] = out.eval_kernel
        finally:
            lib.mm_free_matched(mm.h, C.byref(out))
        sd = synth.Digest()
        got["remaining"] = sd.extract_raw(mm)
        got["state_sha256"] = sd.hexdigest()
        got["active"] = mm.active_count()
        return got
    finally:
        mm.close()
        ts.close()


def _check(name, multi=None):
    g = _golden(name)
    got = _product_pass(g, multi)
    keys = ["groups", "entries", "matched_tickets", "remaining", "active", "groups_sha256", "state_sha256"]
    if g["override"]:
        keys += ["candidates", "candidate_entries", "candidates_sha256"]
    assert {k: got[k] for k in keys} == {k: g[k] for k in keys}, name
    return got


@pytest.mark.parametrize("name", NAMES)
def test_full_size_pass_equals_oracle(name):
    _check(name)


@pytest.mark.parametrize("env", [{"NKM_PIPE": "0"}, {"NKM_GPIPE": "0"}, {"NKM_FAST": "0"}, {"NKM_DENSE": "0"},
                                 {"NKM_KERNEL": "scan"}, {"NKM_THREADS": "4"}, {"NKM_LISTPROOF": "0"},
                                 {"NKM_LISTPROOF": "2"}],
                         ids=["nopipe", "gather-first", "exact-walk", "generic-walk", "scan-kernel", "4-threads",
                              "lists-downloaded", "lists-proof-checked"])
def test_full_size_c3_host_paths(env, monkeypatch):
    """C3 at 1M through the other host replay paths and the chunked scan;
    the hashed scan's lists downloaded although proven (NKM_LISTPROOF=0), and
    downloaded and compared with the proof's claim (2: throws on a miss)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    _check("c3")


def test_full_size_c4_lists_proof_checked(monkeypatch):
    """C4's 64 proven lists at 4M, each downloaded and compared with its
    search's batch rows (NKM_LISTPROOF=2)."""
    monkeypatch.setenv("NKM_LISTPROOF", "2")
    _check("c4")


@pytest.mark.parametrize("env", [{"NKM_RUNS": "0"}, {"NKM_RPACK": "0"}], ids=["row-records", "per-row-lists"])
def test_full_size_c5_host_paths(env, monkeypatch):
    """C5 at 1M with per-row records + merge_rows instead of the run-ordered
    task outputs (NKM_RUNS=0), and with rsmall_kernel's per-row lists instead
    of packed rows (NKM_RPACK=0)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    _check("c5")


POOL_FIELDS = {2: ["properties.region"], 3: ["properties.mode", "properties.region"],
               4: ["properties.mode", "properties.region"], 5: ["properties.bucket"]}


@pytest.mark.parametrize("name,mode", [("c4", "rows"), ("c4", "pools"), ("c3", "pools"), ("c5o", "pools")])
def test_full_size_multi_handle(name, mode):
    """The full-size passes through one multi-device handle (mm_create_multi,
    two sub-handles on device 0): C4 in its BASELINE mode — row-sharded, the
    hashed scan split by candidate chunks between the sub-handles and
    exchanged through host memory, every sub-handle replaying — and with its
    pools placed whole; C3 and C5 + override pool-sharded.  Same digests as
    one oracle pass; C4 rows must run on mscan_hash_kernel (eval_kernel 4)."""
    g = _golden(name)
    m = dict(devices=[0, 0], pool_fields=POOL_FIELDS[g["config"]],
             mode=capi.MM_MULTI_ROWS if mode == "rows" else capi.MM_MULTI_POOLS,
             transport=capi.MM_MULTI_HOST)
    got = _check(name, m)
    if mode == "rows":
        assert got["eval_kernel"] == 4
