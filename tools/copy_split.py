#!/usr/bin/env python3
"""Splits a bench run's copies (rocprofv3 kernel trace + memory-copy trace)
into the Insert hand-over and the pass's own copies.

    rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
        -d <dir> -o run -- python3 bench.py --config 3 --steps S --warmup W
    python3 tools/copy_split.py <dir> --steps S+W > split.json

A step is one Insert() (columns, keyword ids and indexes uploaded to HBM)
followed by one Process() pass (small descriptor uploads right before the
eval kernel, result records and hit lists downloaded right after it).  The
pass's eval kernel (--anchor, one launch per pass) marks each pass: a copy —
a runtime blit kernel (`__amd_rocclr_copyBuffer`, in the kernel trace) or an
SDMA copy (the memory-copy trace, with its direction) — that starts within
--before ms before an anchor's start or --after ms after its end belongs to
that pass; every other copy to the Insert (this trace format carries no byte
counts, so the split is by time).  Per class: copies and device time per step.
"""
import argparse
import bisect
import csv
import glob
import json
import os


def rows(d, suffix):
    for f in sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, required=True, help="steps the bench ran (warmup included)")
    ap.add_argument("--anchor", default="mscan_hash_kernel")
    ap.add_argument("--before", type=float, default=1.0, help="ms before an anchor's start that still belong to its pass")
    ap.add_argument("--after", type=float, default=2.0, help="ms after an anchor's end that still belong to its pass")
    a = ap.parse_args()
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows(a.dir, "kernel_trace.csv")]
    anchors = sorted((s, e) for s, e, n in kern if a.anchor in n)
    starts = [s for s, _ in anchors]
    b_ns, a_ns = a.before * 1e6, a.after * 1e6

    def in_pass(t):
        i = bisect.bisect_right(starts, t)
        if i < len(anchors) and anchors[i][0] - t <= b_ns:  # just before the next anchor
            return True
        return i > 0 and t - anchors[i - 1][1] <= a_ns and t >= anchors[i - 1][0] - b_ns  # during / just after one

    cls = {}

    def add(k, ns):
        c = cls.setdefault(k, [0, 0.0])
        c[0] += 1
        c[1] += ns / 1e6

    for s, e, n in kern:
        if "copyBuffer" in n or "fillBuffer" in n:
            add(("pass" if in_pass(s) else "insert") + "_blit_kernel", e - s)
    for r in rows(a.dir, "memory_copy_trace.csv"):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = "d2h" if "DEVICE_TO_HOST" in r["Direction"] else "h2d" if "HOST_TO_DEVICE" in r["Direction"] else "other"
        add(("pass" if in_pass(s) else "insert") + "_sdma_" + d, e - s)
    out = {"dir": a.dir, "steps": a.steps, "anchor": a.anchor, "anchors": len(anchors),
           "window_ms": [a.before, a.after],
           "per_step": {k: {"copies": round(v[0] / a.steps, 2), "device_ms": round(v[1] / a.steps, 4)}
                        for k, v in sorted(cls.items())}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
