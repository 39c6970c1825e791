#!/usr/bin/env python3
"""The CPU baseline of bench.py's line (BASELINE.md "CPU-baseline plan"),
timed on the host it runs on; bench.py starts it as a child process (the
bench process has initialised the GPU; this one never touches it).

The reference Go/bluge path cannot run here (no Go toolchain),
so the baseline is the oracle (oracle/mm_oracle.cpp: the reference's
per-ticket search, full sort and greedy walk; TEST INFRASTRUCTURE, timed as
the checker, never the product).  Its algorithm class is a FULL SCAN per
search — bluge drives a search from posting lists instead — so two figures
bound the reference from below and from above:

  * full index (the bench's own set): a timed prefix of the pass — the first
    --rows searches over the whole index — extrapolated to the pass by
    sum(c * P * log2 P) over the pass's searches in shrinking pools
    (EXTRAPOLATED, one core);
  * per pool (the cost class of a posting-driven search: each search visits
    its own pool's documents only): every pool's own set in its own process,
    all pools concurrently on min(pools, cores) cores; each times a prefix of
    its pool's pass and extrapolates its pool alone; the all-cores time is the
    slowest pool's, the one-core time their sum (C3: 8 pools, C4: 64; C5's
    buckets of 8 are too small to time apart: full-index prefix only).

    python tools/cpu_baseline.py --config 3 --tickets 1000000 --searches 174983 --matched 999977

`--record c3` instead writes profiles/r03_cpu_full_c3.json from the golden
tests/golden/full_c3.json: whole per-pool oracle passes (NOT extrapolated)
timed by tools/make_full_golden.py on this container's cores — what bench.py
reports as `measured_full_pass`, the calibration of the live figures.
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


def _prefix(config, tickets, rows, pool=None):
    """Times one oracle pass in which only the first `rows` tickets (of the
    pool, or of the whole set) are active; returns (seconds, tickets matched,
    documents in the index)."""
    from nakama_amd import capi, synth
    lib = capi.load_library(os.path.join(ROOT, "oracle", "liboracle_mm.so"))
    ts = synth.TicketSet(config, tickets, first=0, pool_mask=None if pool is None else 1 << pool)
    for k in range(min(rows, ts.n), ts.n):
        ts.tickets[k].intervals = 2  # inactive (Intervals >= MaxIntervals): searched for, never searching
    mm = capi.Matchmaker(lib, max_intervals=2, rev_precision=config in (5, 11), rev_threshold=0)
    try:
        ts.insert_into(mm)
        t0 = time.perf_counter()
        r = mm.process_raw()
        dt = time.perf_counter() - t0
        return dt, sum(len({t for t, _ in g}) for g in r.groups), ts.n
    finally:
        mm.close()
        ts.close()


def _extrapolate(dt, rows, p0, searches, matched):
    """sum over the pass's searches of c * P * log2 P, P the searching
    ticket's remaining pool (shrinking linearly as the pass matches it)."""
    p0 = max(p0, 2.0)
    c = (dt / rows) / (p0 * math.log2(p0))
    steps = max(1, int(round(searches)))
    total = 0.0
    for k in range(steps):
        p = max(2.0, p0 - matched * k / steps)
        total += c * p * math.log2(p)
    return total * searches / steps


def _pool_job(args):
    config, tickets, rows, pool, searches, matched = args
    dt, m, n = _prefix(config, tickets, rows, pool)
    return pool, dt, n, _extrapolate(dt, rows, n, searches, matched)


def record(name):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", f"full_{name}.json")))
    per = g["oracle_pool_pass_s"]
    model, ncpu, usable = host_info()
    out = {"config": g["config"], "tickets": g["tickets"], "pools": len(per), "matched_tickets": g["matched_tickets"],
           "oracle_pool_pass_s": per, "sum_pool_pass_s": round(sum(per), 1), "wall_s": g["wall_s"],
           "cores": 8, "value_one_core": g["matched_tickets"] / sum(per),
           "value_all_cores": g["matched_tickets"] / g["wall_s"], "unit": "tickets/s",
           "host": {"cpu_model": model, "nproc": ncpu, "note": "this build container, 8 oracle processes under nice 10"},
           "sample": (f"MEASURED, not extrapolated: the whole {g['tickets']}-ticket config-{g['config']} pass as "
                      f"{len(per)} per-pool oracle passes (tools/make_full_golden.py {name}), 8 processes on 8 "
                      f"cores; one-core time = the sum of the pool passes, all-cores time = the wall")}
    path = os.path.join(ROOT, "profiles", f"r03_cpu_full_{name}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--record", help="write profiles/r03_cpu_full_<name>.json from the golden's timings")
    ap.add_argument("--config", type=int)
    ap.add_argument("--tickets", type=int)
    ap.add_argument("--searches", type=float, help="searches of the measured GPU pass (whole set)")
    ap.add_argument("--matched", type=float, help="tickets the measured GPU pass matched")
    ap.add_argument("--rows", type=int, default=24)
    ap.add_argument("--pool-rows", type=int, default=64)
    a = ap.parse_args()
    if a.record:
        return record(a.record)
    model, ncpu, usable = host_info()
    out = {"host": {"cpu_model": model, "nproc": ncpu, "usable_cores": usable}, "algorithm": (
        "oracle restatement: one full scan of the index + full sort per search (bluge drives searches from "
        "posting lists: the full-index figure is a lower bound on the reference, the per-pool one closer to it)")}
    npools = N_POOLS.get(a.config, 1)
    # full index, one core
    dt, pre_m, n = _prefix(a.config, a.tickets, a.rows)
    total = _extrapolate(dt, a.rows, a.tickets / npools, a.searches / npools, a.matched / npools) * npools
    out["full_index"] = {
        "value": a.matched / total, "unit": "tickets/s", "cores": 1, "extrapolated_pass_s": total, "prefix_s": dt,
        "sample": (f"EXTRAPOLATED: oracle prefix of the {a.tickets}-ticket config-{a.config} pass ({a.rows} searches "
                   f"over the full index, {dt:.2f} s, {pre_m} tickets matched) scaled by sum(c*P*log2 P) over the "
                   f"pass's {int(a.searches)} searches in {npools} shrinking pools -> {total:.0f} s for "
                   f"{int(a.matched)} matched tickets on one core")}
    if npools > 1:
        workers = max(1, min(npools, usable, 16))
        t0 = time.perf_counter()
        with ProcessPoolExecutor(max_workers=workers) as ex:
            res = list(ex.map(_pool_job, [(a.config, a.tickets, a.pool_rows, p, a.searches / npools,
                                           a.matched / npools) for p in range(npools)]))
        wall = time.perf_counter() - t0
        per = [r[3] for r in res]
        rounds = math.ceil(npools / workers)
        par = max(per) * rounds if rounds > 1 else max(per)
        out["per_pool"] = {
            "value_one_core": a.matched / sum(per), "value_all_cores": a.matched / par, "unit": "tickets/s",
            "cores": workers, "sum_pool_pass_s": sum(per), "parallel_pass_s": par, "timed_wall_s": wall,
            "sample": (f"EXTRAPOLATED per pool, TIMED concurrently: {npools} processes on {workers} cores, each "
                       f"the oracle over its own pool's ~{res[0][2]} tickets timing {a.pool_rows} searches, "
                       f"extrapolated to its pool's pass; all-cores time = slowest pool x {rounds} round(s), "
                       f"one-core time = the sum")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
