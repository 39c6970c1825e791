#!/usr/bin/env python3
"""Headline benchmark: tickets matched/sec and Process() p50 latency at 1M
active tickets (BASELINE.json metric), one interval pass per step.

Workload (BASELINE.json configs[2]): 1,000,000 synthetic
tickets per GPU, party sizes {1:60%,2:20%,3:10%,4:5%,5:5%} (~1.75M presences),
8 pools (mode x region), query = own pool, MinCount=MaxCount=10,
CountMultiple=5, MaxIntervals=2.  A step = insert a fresh ticket set (untimed:
the tickets are resident in HBM before the timed region starts), then ONE
timed LocalMatchmaker.Process() through the C ABI — device searches, the
greedy replay and all post-pass bookkeeping.

Multi-GPU (torchrun, one process per GPU): every rank owns a disjoint ticket
set (its own pools) — the pass partitions by pool with no data-path
collective — so scaling is weak; the timed region of each step is bracketed
by a barrier + device synchronize and the per-step time is the max over ranks.
value = all ranks' matched tickets / sum of per-step max times.

Also reported: roofline of the dominant query-eval kernel of the pass (the
one with the most algorithmic bytes: mscan_kernel on C3; its algorithmic
bytes per launch / its HIP-event launch time, vs 8 TB/s HBM), and the CPU
baseline (the oracle restatement of the reference algorithm, single core,
bounded prefix sample — see DESIGN.md).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
KERNELS = {0: "search_kernel", 1: "scan_kernel", 2: "mscan_kernel"}  # mm_matched.eval_kernel
WORKLOADS = {
    1: "C1: 10k solo 1v1, '+properties.mode:ranked +properties.region:eu'",
    2: "C2: skill-window range queries with ^boost, 1v1",
    3: "C3: 1M tickets/GPU, 5v5 (Min=Max=10, CountMultiple=5), party tickets, 8 pools",
    4: "C4: solo 1v1 over 64 mode x region pools",
    5: "C5: RevPrecision, buckets of 8, Min=2 Max=4 (processDefault; no override registered)",
    7: "C7: regexp / wildcard / fuzzy clauses (blocked lists, alternations, fuzzy map names)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=11)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--tickets", type=int, default=1_000_000, help="tickets per GPU per step")
    ap.add_argument("--cpu-rows", type=int, default=24, help="active rows in the CPU-baseline prefix sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r01_traffic.json"))
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    # torch's HIP runtime comes up before the library's (loading the library
    # first leaves torch with "No HIP GPUs are available")
    import torch
    # NKM_BENCH_BACKEND=gloo rehearses the multi-rank path on a one-GPU box
    # (ranks share device 0; collectives on the host); the driver's runs use
    # "nccl" (RCCL) with one GPU per rank.
    backend = os.environ.get("NKM_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    torch.cuda.synchronize(local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        pg = dist
    return world, rank, local, pg


def barrier_sync(pg, local):
    import torch
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize(local)


def _red_device(pg, local):
    return f"cuda:{local}" if pg.get_backend() == "nccl" else "cpu"


def max_over_ranks(pg, local, x):
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=_red_device(pg, local))
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(pg, local, x):
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=_red_device(pg, local))
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(args):
    """The oracle (oracle/mm_oracle.cpp: per-row full scan + full sort, the
    reference's algorithm class) on one host core: the full 1M-ticket index
    of the same workload, with only the first --cpu-rows tickets active (the
    rest inserted with Intervals = MaxIntervals, i.e. searchable but not
    searching).  Matched tickets / pass wall time."""
    from nakama_amd import capi, synth
    lib = capi.load_library(os.path.join(ROOT, "oracle", "liboracle_mm.so"))
    ts = synth.TicketSet(args.config, args.tickets, first=0)
    for k in range(args.cpu_rows, ts.n):
        ts.tickets[k].intervals = 2
    mm = capi.Matchmaker(lib, max_intervals=2)
    try:
        ts.insert_into(mm)
        t0 = time.perf_counter()
        r = mm.process_raw()
        dt = time.perf_counter() - t0
        matched = sum(len({t for t, _ in g}) for g in r.groups)
    finally:
        mm.close()
        ts.close()
    return {"value": matched / dt if dt > 0 else 0.0, "unit": "tickets/s", "cores": 1, "kind": "port",
            "sample": f"oracle pass over the full {args.tickets}-ticket config-{args.config} index with the first "
                      f"{args.cpu_rows} tickets active: {matched} tickets matched in {dt:.2f} s "
                      f"({dt / max(1, args.cpu_rows) * 1e3:.0f} ms per searching ticket)",
            "pass_s": dt, "matched": matched}


def main():
    args = parse()
    world, rank, local, pg = dist_setup(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    import nakama_amd
    from nakama_amd import synth

    mm = nakama_amd.LocalMatchmaker(max_intervals=2, device=local, rev_precision=args.config == 5)
    # Pool sharding (weak scaling): the N-GPU workload is N disjoint instances
    # of the config's pool set (region values suffixed per instance, so C3's
    # 8 pools become 8N), and GPU r owns instance r whole — every GPU runs
    # exactly the single-GPU workload, no ticket can match across GPUs, and
    # the pass needs no data-path collective.
    times, matched_all, presences_all, ins_times = [], [], [], []
    eval_ms = eval_bytes = launches = 0
    batches, kernels = [], set()
    for step in range(args.warmup + args.steps):
        first = (step * world + rank) * args.tickets
        ts = (synth.TicketSet(args.config, args.tickets, first=first, shard=rank) if world > 1
              else synth.TicketSet(args.config, args.tickets, first=first))
        t_ins = time.perf_counter()
        ts.insert_into(mm)  # untimed: one Insert() C-ABI call (store maintenance, index build, H2D upload)
        ins_dt = time.perf_counter() - t_ins
        barrier_sync(pg, local)
        t0 = time.perf_counter()
        out = mm.process_call()  # the C-ABI call: one whole Process() pass
        barrier_sync(pg, local)
        dt = time.perf_counter() - t0
        n_groups, matched, pres, r = mm.process_summary(out)  # untimed: counts the groups, frees them
        ts.close()
        dt_max = max_over_ranks(pg, local, dt)
        if step >= args.warmup:
            times.append(dt_max)
            ins_times.append(max_over_ranks(pg, local, ins_dt))
            matched_all.append(sum_over_ranks(pg, local, matched))
            presences_all.append(sum_over_ranks(pg, local, pres))
            eval_ms += r.eval_ms
            eval_bytes += r.eval_bytes
            launches += r.eval_launches
            batches.append(r.n_batches)
            kernels.add(KERNELS.get(r.eval_kernel, str(r.eval_kernel)))
        # drain what is left so the next step starts from a fresh 1M set
        mm.Remove([t.ticket for t in mm.Extract()]) if mm.ticket_count() else None
    total_t = sum(times)
    value = sum(matched_all) / total_t
    achieved = (eval_bytes / 1e9) / (eval_ms / 1e3) if eval_ms > 0 else 0.0
    avg_launch_ms = eval_ms / max(1, launches)
    # HBM bytes per launch from the PMC passes (tools/pmc_traffic.py), when
    # they were taken on this kernel
    traffic = None
    if os.path.exists(args.traffic):
        try:
            tr = json.load(open(args.traffic))
            if tr.get("kernel") in kernels:
                traffic = tr.get("bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": "tickets matched/sec + Process() interval p50 latency at 1M active tickets",
        "value": value,
        "unit": "tickets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * total_t / args.steps,
        "p50_ms": 1e3 * statistics.median(times),
        "presences_per_s": sum(presences_all) / total_t,
        # the host-to-HBM hand-over: the Insert() call that precedes each pass
        # (not part of value: inputs are resident when the timed region starts)
        "insert_ms": 1e3 * statistics.median(ins_times),
        "with_insert_tickets_per_s": sum(matched_all) / (total_t + sum(ins_times)),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64/f64",
        "data": "synthetic",
        "config": {"workload": WORKLOADS.get(args.config, str(args.config)), "tickets_per_gpu": args.tickets,
                   "max_intervals": 2, "parallelism": f"pool-sharded x{world}: {world} disjoint pool sets, one per GPU",
                   "matched_per_step": sum(matched_all) / args.steps, "batches_per_pass": batches},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "+".join(sorted(kernels)), "launches": launches, "avg_launch_ms": avg_launch_ms,
                     "bytes_per_launch": eval_bytes / max(1, launches)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(args)
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
    else:
        out["cpu_baseline"] = None
    mm.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.barrier()
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
