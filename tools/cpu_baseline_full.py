#!/usr/bin/env python3
"""Full (not extrapolated) oracle passes for the configs small enough to run
whole on one core, as BASELINE.md asks for C1 and C2: the oracle restatement
(oracle/mm_oracle.cpp — the reference's per-ticket search, sort and greedy
walk) inserts the config's synthetic set and runs ONE Process() pass; the line
records the pass time, the matched tickets and tickets/s, with the host CPU.

    python tools/cpu_baseline_full.py --config 1 --tickets 10000 --out profiles/r02_cpu_c1.json

CPU-only (test infrastructure: the oracle is the checker, never the product).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--tickets", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    from nakama_amd import capi, synth
    import bench
    lib = capi.load_library(os.path.join(ROOT, "oracle", "liboracle_mm.so"))
    ts = synth.TicketSet(a.config, a.tickets, first=0)
    mm = capi.Matchmaker(lib, max_intervals=2, rev_precision=a.config == 5, rev_threshold=0)
    try:
        t0 = time.perf_counter()
        ts.insert_into(mm)
        t_ins = time.perf_counter() - t0
        t0 = time.perf_counter()
        r = mm.process_raw()
        dt = time.perf_counter() - t0
        matched = sum(len({t for t, _ in g}) for g in r.groups)
        presences = sum(len(g) for g in r.groups)
    finally:
        mm.close()
        ts.close()
    model, ncpu, usable = bench.host_info()
    out = {"config": a.config, "workload": bench.WORKLOADS.get(a.config), "tickets": a.tickets,
           "kind": "port", "cores": 1, "insert_s": t_ins, "pass_s": dt, "groups": len(r.groups),
           "matched_tickets": matched, "matched_presences": presences, "value": matched / dt, "unit": "tickets/s",
           "host": {"cpu_model": model, "nproc": ncpu, "usable_cores": usable},
           "note": "one whole oracle Process() pass on one core (not extrapolated)"}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
