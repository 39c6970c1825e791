#!/usr/bin/env python3
"""Per-launch HBM traffic of a query-eval kernel from rocprofv3 PMC passes.

Inputs (one rocprofv3 run per counter, as MI355X_MICROARCH.md prescribes):
  --fetch  <dir>   counter_collection.csv of `--pmc FETCH_SIZE -- python3 bench.py ...`
  --write  <dir>   counter_collection.csv of `--pmc WRITE_SIZE -- python3 bench.py ...`
  --calib-fetch / --calib-write <dir>  the same counters over tools/fetch_calib
                                        (known byte counts per access width)

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 tallies a wide coalesced read at
half its bytes (guide, HBM section); other widths are calibrated here: the
correction for a kernel is  known_bytes / counter  of the calibration kernel
with search_kernel's dominant access width (4-B/lane posting-list loads and
4/8-B column gathers -> the u32 stream row).  Output: JSON with the raw and
corrected bytes per launch; bench.py reports `bytes_per_launch` as
roofline.traffic.
"""
import argparse
import csv
import glob
import json
import os
import statistics

CALIB_BYTES = 1 << 30
# launch order of tools/fetch_calib.hip
CALIB_READ = ["read_v16", "read_u64", "read_u32", "read_u8", "read_stride8_u32"]
CALIB_WRITE = ["write_v16", "write_u64", "write_u32", "write_u8"]


def rows(d, counter):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter:
                    out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    out.sort()
    return out


def calib(d, counter, names, kernel_filter):
    rs = [r for r in rows(d, counter) if kernel_filter in r[1]]
    got = {}
    for name, r in zip(names, rs):
        got[name] = {"counter_bytes": r[2], "factor": CALIB_BYTES / r[2] if r[2] else None}
    return got


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib-fetch")
    ap.add_argument("--calib-write")
    ap.add_argument("--kernel", default="mscan_kernel")
    ap.add_argument("--out", required=True)
    ap.add_argument("--config", type=int, required=True, help="bench.py --config of the profiled run")
    ap.add_argument("--tickets", type=int, required=True, help="bench.py --tickets of the profiled run")
    a = ap.parse_args()

    fetch = [r[2] for r in rows(a.fetch, "FETCH_SIZE") if a.kernel in r[1]]
    write = [r[2] for r in rows(a.write, "WRITE_SIZE") if a.kernel in r[1]]
    # bench.py attaches this file only to a line of the same kernel, config and size
    res = {"kernel": a.kernel, "config": a.config, "tickets": a.tickets,
           "launches_fetch": len(fetch), "launches_write": len(write),
           "fetch_raw_bytes_per_launch": statistics.mean(fetch) if fetch else None,
           "write_raw_bytes_per_launch": statistics.mean(write) if write else None}
    ff, wf = 2.0, 1.0  # the guide's gfx950 corrections when no calibration is given
    if a.calib_fetch:
        c = calib(a.calib_fetch, "FETCH_SIZE", CALIB_READ, "read_")
        res["calib_fetch"] = c
        if c.get("read_u32", {}).get("factor"):
            ff = c["read_u32"]["factor"]
    if a.calib_write:
        c = calib(a.calib_write, "WRITE_SIZE", CALIB_WRITE, "write_")
        res["calib_write"] = c
        if c.get("write_v16", {}).get("factor"):
            wf = c["write_v16"]["factor"]  # DHit stores are 16 B per lane
    res["fetch_factor"] = ff
    res["write_factor"] = wf
    if fetch and write:
        res["bytes_per_launch"] = ff * res["fetch_raw_bytes_per_launch"] + wf * res["write_raw_bytes_per_launch"]
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
