#!/usr/bin/env python3
"""The CPU baseline of bench.py's line (BASELINE.md "CPU-baseline plan"),
timed on the host it runs on; bench.py starts it as a child process (the
bench process has initialised the GPU; this one never touches it).

The reference Go/bluge path cannot run here (no Go toolchain),
so the baseline is the oracle (oracle/mm_oracle.cpp: the reference's
per-ticket search, sort order and greedy walk; TEST INFRASTRUCTURE, timed as
the checker, never the product): kind "port".

Cost model of one oracle search (search_hits_walk): it visits every document
of its index (N_all, dead ones included: bluge's deleted documents stay until
a merge) and heaps its H hits, then pops the few the walk reads —
    t = a * N_all + b * H.
A pool pass of S searches whose pool loses M of its N tickets as the pass
matches them (linearly) therefore costs S * (a * N + b * (N - M / 2)).  `a`
and `b` are measured per pool from two short prefixes of the pool's own pass
(the first R rows searching): one over the whole pool (H = N), one after half
its tickets were removed (H = N / 2, still N documents visited).  The model is
checked against whole measured per-pool passes of the same oracle
(tools/make_full_golden.py timings: profiles/r04_cpu_full_<c>.json,
`--calibrate`).

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

N_POOLS = {3: 8, 4: 64}
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


def _prefix(config, tickets, rows, pool, remove_half):
    """One oracle pass of `pool`'s tickets in which only the first `rows`
    search (the others inactive: Intervals >= MaxIntervals, searched for but
    never searching); with remove_half every other inactive ticket is removed
    first (its document stays in the index, visited but never a hit).
    Returns (seconds per search, documents visited per search, hits)."""
    from nakama_amd import capi, synth
    ts = synth.TicketSet(config, tickets, first=0, pool_mask=1 << pool)
    for k in range(min(rows, ts.n), ts.n):
        ts.tickets[k].intervals = 2
    mm = capi.Matchmaker(_oracle(), max_intervals=2, rev_precision=config in (5, 11), rev_threshold=0)
    try:
        ts.insert_into(mm)
        n = ts.n
        if remove_half:
            mm.Remove([ts.ticket_id(k) for k in range(rows, ts.n, 2)])
        h = mm.ticket_count()
        t0 = time.perf_counter()
        mm.process_raw()
        dt = time.perf_counter() - t0
        return dt / max(1, min(rows, n)), n, h
    finally:
        mm.close()
        ts.close()


def _pool_model(args):
    """(pool, N, a, b): the pool's per-search cost coefficients."""
    config, tickets, rows, pool = args
    t1, n, h1 = _prefix(config, tickets, rows, pool, False)
    t2, _, h2 = _prefix(config, tickets, rows, pool, True)
    b = max(0.0, (t1 - t2) / max(1, h1 - h2))
    a = max(0.0, (t1 - b * h1) / n)
    return pool, n, a, b, t1, t2


def pool_pass_s(n, a, b, searches, matched):
    return searches * (a * n + b * (n - matched / 2.0))


def per_pool(config, tickets, rows, searches, matched, workers):
    npools = N_POOLS[config]
    t0 = time.perf_counter()
    with ProcessPoolExecutor(max_workers=workers) as ex:
        res = list(ex.map(_pool_model, [(config, tickets, rows, p) for p in range(npools)]))
    wall = time.perf_counter() - t0
    per = [pool_pass_s(n, a, b, searches / npools, matched / npools) for _, n, a, b, _, _ in res]
    return res, per, wall


def c5_chunks(config, tickets, chunks):
    """Whole passes of `chunks` 1000-ticket chunks spread over the set."""
    from nakama_amd import capi, synth
    nch = tickets // C5_CHUNK
    picks = sorted({(nch * i) // chunks for i in range(chunks)})
    total, matched = 0.0, 0
    for c in picks:
        ts = synth.TicketSet(config, C5_CHUNK, first=c * C5_CHUNK)
        mm = capi.Matchmaker(_oracle(), max_intervals=2, rev_precision=True, rev_threshold=0)
        try:
            ts.insert_into(mm)
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
    res, per, wall = per_pool(config, tickets, rows, searches, g["matched_tickets"], workers)
    meas = full["oracle_pool_pass_s"]
    ratio = [p / m for p, m in zip(per, meas)]
    out = {"config": config, "tickets": tickets, "pools": npools, "prefix_rows": rows,
           "model_pool_pass_s": [round(x, 1) for x in per], "measured_pool_pass_s": meas,
           "model_over_measured": {"min": min(ratio), "max": max(ratio), "sum": sum(per) / sum(meas)},
           "coefficients": [{"pool": p, "N": n, "a_ns": a * 1e9, "b_ns": b * 1e9} for p, n, a, b, _, _ in res],
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
    ap.add_argument("--pool-rows", type=int, default=48)
    ap.add_argument("--chunks", type=int, default=1000, help="C5: chunk passes timed (all 1000: the whole pass)")
    a = ap.parse_args()
    model, ncpu, usable = host_info()
    workers = max(1, min(usable, 16))
    if a.record:
        return record(a.record)
    if a.calibrate:
        return calibrate(a.calibrate, a.pool_rows, workers)
    out = {"host": {"cpu_model": model, "nproc": ncpu, "usable_cores": usable}, "algorithm": (
        "oracle restatement (port): per search a visit of every document of its index + a heap of the hits in "
        "the reference's sort order; searches visit their own pool's index (the cost class of bluge's posting-"
        "driven search), C5 its 1000-ticket chunk")}
    if a.config in N_POOLS:
        npools = N_POOLS[a.config]
        w = max(1, min(npools, workers))
        res, per, wall = per_pool(a.config, a.tickets, a.pool_rows, a.searches, a.matched, w)
        rounds = math.ceil(npools / w)
        par = max(per) * rounds if rounds > 1 else max(per)
        out["value"] = a.matched / sum(per)
        out["cores"] = 1
        out["sample"] = (f"EXTRAPOLATED per pool (model t = a*N_all + b*H per search, a and b from two {a.pool_rows}-"
                         f"row prefixes of each pool's own pass, TIMED concurrently on {w} cores; "
                         f"profiles/r04_cpu_calib_c*.json checks it against measured whole passes): "
                         f"{npools} pools of ~{res[0][1]} tickets, one-core time = sum of the pools' passes "
                         f"{sum(per):.0f} s")
        out["all_cores"] = {"value": a.matched / par, "cores": w,
                            "note": f"the slowest pool's pass x {rounds} round(s) = {par:.0f} s"}
        out["model"] = {"a_ns": [round(r[2] * 1e9, 2) for r in res], "b_ns": [round(r[3] * 1e9, 2) for r in res],
                        "timed_wall_s": round(wall, 1)}
    else:
        t, m, k, nch = c5_chunks(a.config, a.tickets, a.chunks)
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
