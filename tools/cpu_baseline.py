#!/usr/bin/env python3
"""The CPU baseline of bench.py's line (BASELINE.md "CPU-baseline plan"),
timed on the host it runs on; bench.py starts it as a child process (the
bench process has initialised the GPU; this one never touches it).

The reference Go/bluge path cannot run here (no Go toolchain),
so the baseline is the oracle (oracle/mm_oracle.cpp: the reference's
per-ticket search, sort order and greedy walk; TEST INFRASTRUCTURE, timed as
the checker, never the product): kind "port".

Cost of one oracle search (search_hits_walk): a visit of every document of
its index and a heap of its H live hits, then the few pops the walk reads.
H falls as the pass matches tickets, and so does the live working set the
visit touches (the matched tickets are the earliest-created: the rows search
in created order and take the earliest partners), so the per-search cost is
SAMPLED along the pass: with the pool's first m tickets removed (the pass's
state once m tickets are matched: removed and matched documents are both
dead) the next R rows search, at m = 0, M/4, M/2, 3M/4 and M - R for a pool
that matches M tickets; the pool's pass = its searches x the trapezoid mean
of the five per-search times.  The model is checked against whole measured
per-pool passes of the same oracle (tools/make_full_golden.py timings:
profiles/r04_cpu_full_<c>.json, `--calibrate`).

  * C3 / C4: every pool in its own process, all pools concurrently on
    min(pools, cores) cores; one-core time = the sum of the pools' passes,
    all-cores time = the slowest pool x the rounds (C4 "per-pool
    passes ... sum and per-core parallel time");
  * C5 (buckets of 8): the pass is the concatenation of independent
    1000-ticket chunks (125 whole buckets; tools/make_full_golden.py c5):
    --chunks chunk passes are TIMED whole and the pass extrapolated linearly
    by the chunk count ("prefix + extrapolation").

    python tools/cpu_baseline.py --config 3 --tickets 1000000 --searches 174983 --matched 999977
    python tools/cpu_baseline.py --record c4        # measured passes -> profiles/r04_cpu_full_c4.json
    python tools/cpu_baseline.py --calibrate c4     # the model vs those measured passes
"""
import argparse
import json
import math
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_POOLS = {2: 4, 3: 8, 4: 64}
# searching rows per sample: enough searches for a stable per-search time
# (C3: ~10 rows per group; C2 / C4: 2)
POOL_ROWS = {2: 200, 3: 400, 4: 100}
C5_CHUNK = 1000


def host_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return model, os.cpu_count(), usable


def _oracle():
    from nakama_amd import capi
    return capi.load_library(os.path.join(ROOT, "oracle", "liboracle_mm.so"))


def _prefix(config, tickets, rows, pool, skip):
    """One oracle pass of `pool`'s tickets with its first `skip` tickets
    removed, in which the next `rows` search (the later ones inactive:
    Intervals >= MaxIntervals, searched for but never searching).  Returns
    (seconds per search, live documents).  A search is a row that was not
    selected before its turn: the group makers plus the rows that searched
    and matched nothing."""
    from nakama_amd import capi, synth
    ts = synth.TicketSet(config, tickets, first=0, pool_mask=1 << pool)
    n = ts.n
    skip = max(0, min(skip, n - 1))
    for k in range(min(skip + rows, n), n):
        ts.tickets[k].intervals = 2
    mm = capi.Matchmaker(_oracle(), max_intervals=2, rev_precision=config in (5, 11), rev_threshold=0)
    try:
        ts.insert_into(mm)
        if skip:
            mm.Remove([ts.ticket_id(k) for k in range(skip)])
        h = mm.ticket_count()
        t0 = time.perf_counter()
        r = mm.process_raw()
        dt = time.perf_counter() - t0
        active = {ts.ticket_id(k) for k in range(skip, min(skip + rows, n))}
        grouped = {t for g in r.groups for t, _ in g}
        searches = len(r.groups) + len(active - grouped)
        return dt / max(1, searches), h
    finally:
        mm.close()
        ts.close()


SAMPLES = 5  # points along the pass (m = 0, M/4, M/2, 3M/4, M - R)


def _sample(args):
    config, tickets, rows, pool, k, m_pool = args
    skip = int(round(m_pool * k / (SAMPLES - 1))) if k < SAMPLES - 1 else int(m_pool) - rows
    t, h = _prefix(config, tickets, rows, pool, max(0, skip))
    return pool, k, t, h


def pool_pass_s(ts, searches):
    """searches x the trapezoid mean of the per-search times sampled at equal steps of the pass"""
    mean = (sum(ts) - (ts[0] + ts[-1]) / 2.0) / (len(ts) - 1)
    return searches * mean


def per_pool(config, tickets, rows, searches, matched, workers):
    npools = N_POOLS[config]
    m_pool = matched / npools
    t0 = time.perf_counter()
    jobs = [(config, tickets, rows, p, k, m_pool) for p in range(npools) for k in range(SAMPLES)]
    with ProcessPoolExecutor(max_workers=workers) as ex:
        res = list(ex.map(_sample, jobs))
    wall = time.perf_counter() - t0
    t = [[0.0] * SAMPLES for _ in range(npools)]
    h = [[0] * SAMPLES for _ in range(npools)]
    for p, k, tk, hk in res:
        t[p][k] = tk
        h[p][k] = hk
    per = [pool_pass_s(t[p], searches / npools) for p in range(npools)]
    return t, h, per, wall


def c5_chunks(config, tickets, chunks, override=False):
    """Whole passes of `chunks` 1000-ticket chunks spread over the set.
    override: the pass is processCustom's candidate pass, the bench's native
    first-disjoint override (tools/synth.cpp) and mm_process_commit — the
    same step bench.py --override times on the GPU."""
    from nakama_amd import capi, synth
    nch = tickets // C5_CHUNK
    picks = sorted({(nch * i) // chunks for i in range(chunks)})
    total, matched = 0.0, 0
    for c in picks:
        ts = synth.TicketSet(config, C5_CHUNK, first=c * C5_CHUNK)
        mm = capi.Matchmaker(_oracle(), max_intervals=2, rev_precision=True, rev_threshold=0,
                             override=(lambda g: g) if override else None)
        try:
            ts.insert_into(mm)
            if override:
                t0 = time.perf_counter()
                out = mm.process_call()
                if out.is_candidates:
                    out = synth.override_commit(mm, out)
                total += time.perf_counter() - t0
                matched += mm.process_summary(out)[1]
            else:
                t0 = time.perf_counter()
                r = mm.process_raw()
                total += time.perf_counter() - t0
                matched += sum(len({t for t, _ in g}) for g in r.groups)
        finally:
            mm.close()
            ts.close()
    return total, matched, len(picks), nch


def record(name):
    """profiles/r04_cpu_full_<name>.json: the whole per-pool oracle passes
    tools/make_full_golden.py timed (MEASURED, not extrapolated)."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", f"full_{name}.json")))
    per = g["oracle_pool_pass_s"]
    model, ncpu, usable = host_info()
    out = {"config": g["config"], "tickets": g["tickets"], "pools": len(per), "matched_tickets": g["matched_tickets"],
           "oracle_pool_pass_s": per, "sum_pool_pass_s": round(sum(per), 1), "wall_s": g["wall_s"],
           "cores": g.get("jobs", 7), "value_one_core": g["matched_tickets"] / sum(per),
           "value_all_cores": g["matched_tickets"] / g["wall_s"], "unit": "tickets/s",
           "host": {"cpu_model": model, "nproc": ncpu, "note": "this build container"},
           "sample": (f"MEASURED, not extrapolated: the whole {g['tickets']}-ticket config-{g['config']} pass as "
                      f"{len(per)} per-pool oracle passes (tools/make_full_golden.py {name}) on "
                      f"{g.get('jobs', 7)} cores; one-core time = the sum of the pool passes, all-cores time = "
                      f"the wall")}
    path = os.path.join(ROOT, "profiles", f"r04_cpu_full_{name}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)


def calibrate(name, rows, workers):
    """The per-pool model against the measured passes of the same oracle:
    profiles/r04_cpu_calib_<name>.json."""
    full = json.load(open(os.path.join(ROOT, "profiles", f"r04_cpu_full_{name}.json")))
    g = json.load(open(os.path.join(ROOT, "tests", "golden", f"full_{name}.json")))
    config, tickets = g["config"], g["tickets"]
    npools = N_POOLS[config]
    searches = g["groups"] + g["remaining"]  # rows that searched: the group makers and the leftovers
    t, h, per, wall = per_pool(config, tickets, rows, searches, g["matched_tickets"], workers)
    meas = full["oracle_pool_pass_s"]
    ratio = [p / m for p, m in zip(per, meas)]
    out = {"config": config, "tickets": tickets, "pools": npools, "prefix_rows": rows, "workers": workers,
           "model_pool_pass_s": [round(x, 1) for x in per], "measured_pool_pass_s": meas,
           "model_over_measured": {"min": min(ratio), "max": max(ratio), "sum": sum(per) / sum(meas)},
           "per_search_ms": [[round(x * 1e3, 3) for x in tp] for tp in t], "live_docs": h,
           "timed_wall_s": wall, "host": dict(zip(("cpu_model", "nproc", "usable"), host_info()))}
    path = os.path.join(ROOT, "profiles", f"r04_cpu_calib_{name}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["model_over_measured"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--record", help="write profiles/r04_cpu_full_<name>.json from the golden's timings")
    ap.add_argument("--calibrate", help="the model against profiles/r04_cpu_full_<name>.json")
    ap.add_argument("--config", type=int)
    ap.add_argument("--tickets", type=int)
    ap.add_argument("--searches", type=float, help="searches of the measured GPU pass (whole set)")
    ap.add_argument("--matched", type=float, help="tickets the measured GPU pass matched")
    ap.add_argument("--pool-rows", type=int, default=0, help="searching rows per sample (default POOL_ROWS)")
    ap.add_argument("--chunks", type=int, default=1000, help="C5: chunk passes timed (all 1000: the whole pass)")
    ap.add_argument("--override", action="store_true", help="C5: with the MatchmakerOverride hand-off (bench --override)")
    ap.add_argument("--workers", type=int, default=0, help="concurrent pool processes (default: the usable cores, <= 16)")
    a = ap.parse_args()
    model, ncpu, usable = host_info()
    workers = a.workers or max(1, min(usable, 16))
    if a.record:
        return record(a.record)
    if a.calibrate:
        cfg = json.load(open(os.path.join(ROOT, "tests", "golden", f"full_{a.calibrate}.json")))["config"]
        return calibrate(a.calibrate, a.pool_rows or POOL_ROWS[cfg], workers)
    out = {"host": {"cpu_model": model, "nproc": ncpu, "usable_cores": usable}, "algorithm": (
        "oracle restatement (port): per search a visit of every document of its index + a heap of the hits in "
        "the reference's sort order; searches visit their own pool's index (the cost class of bluge's posting-"
        "driven search), C5 its 1000-ticket chunk")}
    if a.config in N_POOLS:
        npools = N_POOLS[a.config]
        w = max(1, min(npools, workers))
        rows = a.pool_rows or POOL_ROWS[a.config]
        t, h, per, wall = per_pool(a.config, a.tickets, rows, a.searches, a.matched, w)
        rounds = math.ceil(npools / w)
        par = max(per) * rounds if rounds > 1 else max(per)
        out["value"] = a.matched / sum(per)
        out["cores"] = 1
        out["sample"] = (f"EXTRAPOLATED per pool: per-search times SAMPLED at {SAMPLES} points of each pool's own "
                         f"pass ({rows} searching rows each, the earlier-matched tickets removed), TIMED "
                         f"concurrently on {w} cores, pass = searches x their trapezoid mean "
                         f"(profiles/r04_cpu_calib_c*.json checks it against measured whole passes): {npools} pools "
                         f"of ~{h[0][0]} tickets, one-core time = sum of the pools' passes {sum(per):.0f} s")
        out["all_cores"] = {"value": a.matched / par, "cores": w,
                            "note": f"the slowest pool's pass x {rounds} round(s) = {par:.0f} s"}
        out["model"] = {"per_search_ms_pool0": [round(x * 1e3, 3) for x in t[0]], "timed_wall_s": round(wall, 1)}
    else:
        t, m, k, nch = c5_chunks(a.config, a.tickets, a.chunks, a.override)
        if a.override:
            out["algorithm"] += ("; + MatchmakerOverride: processCustom's candidates (combineIndexes), the native "
                                 "first-disjoint override and mm_process_commit, as bench.py --override")
        total = t * nch / k
        out["value"] = a.matched / total
        out["cores"] = 1
        out["sample"] = ((f"MEASURED: the whole {a.tickets}-ticket pass as its {nch} chunk passes of {C5_CHUNK} "
                          f"tickets (125 buckets each), {t:.1f} s for {m} matched on one core") if k == nch else
                         (f"EXTRAPOLATED: {k} whole chunk passes of {C5_CHUNK} tickets (125 buckets each) TIMED, "
                          f"{t:.2f} s for {m} matched, scaled by the {nch} chunks -> {total:.0f} s for the "
                          f"{a.tickets}-ticket pass on one core"))
        if k == nch:
            out["value"] = m / t
        out["all_cores"] = {"value": a.matched / (total / workers), "cores": workers,
                            "note": "independent chunks over the cores (linear)"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
