#!/usr/bin/env python3
"""The pool-sharded cluster merge (mm_merge_positions_ex, mm_cluster.cpp) in
one process: world ranks' ascending CreatedAt keys (C3's volume: 175k groups
per rank at world 8), every rank's positions computed in turn; prints one
JSON line of per-rank medians.  LOCAL_WORLD_SIZE sets the merge pool's
threads (the process's CPUs over it, at most 8), as under torchrun."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nakama_amd import cluster  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--groups", type=int, default=175_000)
ap.add_argument("--reps", type=int, default=21)
a = ap.parse_args()
L = cluster.router_lib()
rng = np.random.default_rng(1)
n, world = a.groups, a.world
ks = [np.sort(rng.choice(np.arange(4 * n, dtype=np.int64), n, replace=False)) * world + r for r in range(world)]
allk = np.concatenate(ks)
counts = np.full(world, n, dtype=np.int32)
flat = np.sort(allk)
out = {"world": world, "groups_per_rank": n, "local_world_size": os.environ.get("LOCAL_WORLD_SIZE"),
       "cpu": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?"),
       "cpus": len(os.sched_getaffinity(0))}
for sorted_flag, name in ((1, "sorted_ms"), (0, "checked_ms")):
    per_rank = []
    for rank in range(world):
        pos = np.zeros(n, dtype=np.int64)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            L.mm_merge_positions_ex(allk.ctypes.data, n, counts.ctypes.data, world, rank, sorted_flag, pos.ctypes.data)
            ts.append(1e3 * (time.perf_counter() - t0))
        assert np.array_equal(flat[pos], ks[rank])
        per_rank.append(statistics.median(ts))
    out[name] = {"median_over_ranks": statistics.median(per_rank), "max_over_ranks": max(per_rank)}
print(json.dumps(out))
