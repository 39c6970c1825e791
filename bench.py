#!/usr/bin/env python3
"""Headline benchmark: tickets matched/sec and Process() p50 latency at 1M
active tickets (BASELINE.json metric), one interval pass per step.

Workload (BASELINE.json configs[2]): 1,000,000 synthetic
tickets per GPU, party sizes {1:60%,2:20%,3:10%,4:5%,5:5%} (~1.75M presences),
8 pools (mode x region) per GPU, query = own pool, MinCount=MaxCount=10,
CountMultiple=5, MaxIntervals=2.  A step = insert a fresh ticket set
(untimed: the tickets are resident in HBM before the timed region starts),
then ONE timed Process() through the C ABI — device searches, the greedy
replay and all post-pass bookkeeping.

Multi-GPU (torchrun, one process per GPU, RCCL): ONE ticket set of N x 1M
tickets over 8N pools (C3's pools times N, every pool spread over the whole
index range) goes through the product's multi-GPU front
(nakama_amd/cluster.py): each rank ingests a 1M slice, the front routes every
ticket to its pool's rank (routing keys + one all-to-all of packed records,
untimed like the single-GPU insert), and the timed step is the cluster-wide
Process(): every rank's pass plus the merge of the ranks' group lists into the
reference's group order (an all-gather of 8 B per group, merged on rank 0).
Scaling is weak for C3 (1M per GPU); --config 4 (4M tickets over 64 pools in
total) and --config 5 (1M in total) split one fixed set (strong).  Each step is
bracketed by a barrier + device synchronize; its time is the max over ranks;
value = all ranks' matched tickets / sum of the per-step max times.

Also reported: roofline of the dominant query-eval kernel of the pass (the
one with the most algorithmic bytes: mscan_kernel on C3; algorithmic bytes per
launch / its HIP-event launch time, vs 8 TB/s HBM) with the PMC traffic of the
same kernel from the committed rocprofv3 pass, and the CPU baseline (the
oracle restatement of the reference algorithm: a timed prefix of the 1M pass,
extrapolated to the whole pass as BASELINE.md prescribes — see cpu_baseline).
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
KERNELS = {0: "search_kernel", 1: "scan_kernel", 2: "mscan_kernel", 3: "rsmall_kernel", 4: "mscan_hash_kernel",
           5: "rpack_kernel", 6: "rsrc_merge_kernel", 7: "rsrc_tile_kernel"}  # mm_matched.eval_kernel
WORKLOADS = {
    1: "C1: 10k solo 1v1, '+properties.mode:ranked +properties.region:eu'",
    2: "C2: skill-window range queries with ^boost, 1v1",
    3: "C3: 1M tickets/GPU, 5v5 (Min=Max=10, CountMultiple=5), party tickets, 8 pools/GPU",
    4: "C4: solo 1v1, 4M tickets over 64 mode x region pools (in total)",
    5: "C5: RevPrecision, buckets of 8, Min=2 Max=4, 1M in total",
    7: "C7: regexp / wildcard / fuzzy clauses (blocked lists, alternations, fuzzy map names)",
    11: "C5 with buckets of 64 (63 filtered hits per row: processCustom's combineIndexes hands over no candidate, "
        "matchmaker_process.go:588), RevPrecision, Min=2 Max=4, 1M in total",
}
# the query fields a pool is keyed on (the cluster front's routing)
POOL_FIELDS = {1: ("properties.mode", "properties.region"), 2: ("properties.region",),
               3: ("properties.mode", "properties.region"),
               4: ("properties.mode", "properties.region"), 5: ("properties.bucket",), 11: ("properties.bucket",)}
# BASELINE.json configs: C1 10k, C2 100k, C4 4M in total; the others 1M (per GPU for C3)
DEFAULT_TICKETS = {1: 10_000, 2: 100_000, 4: 4_000_000}
STRONG = (4, 5, 11)               # configs whose ticket count is the whole job's
REV = (5, 11)                     # RevPrecision configs


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=11)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--tickets", type=int, default=None,
                    help="tickets per GPU per step (C3), or in total (C4, C5); default 1M (C4: 4M)")
    ap.add_argument("--cpu-rows", type=int, default=24, help="active rows in the CPU-baseline prefix sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="do not bind the process to its GPU's NUMA node (one process per GPU)")
    ap.add_argument("--no-deliver", dest="deliver", action="store_false",
                    help="time mm_process alone and free its result untimed, instead of the default pipelined "
                         "delivery (BASELINE.md: the pass includes delivery to a no-op router): mm_set_delivery + "
                         "mm_process_deliver, the timed step ending when the pass's result is handed to the "
                         "library's delivery thread, whose callback is a native no-op router (tools/synth.cpp "
                         "synth_deliver_noop: every entry read, tickets counted) running behind the step; its time and "
                         "the flush wait after the step are reported beside the line (single GPU, processDefault; "
                         "the cluster front and the override path time mm_process)")
    ap.add_argument("--override", action="store_true",
                    help="register a MatchmakerOverride (processCustom path): the timed step is the candidate pass, "
                         "a native first-disjoint override and mm_process_commit (per rank under the cluster front)")
    ap.add_argument("--multi-handle", type=int, default=0, metavar="N",
                    help="one process drives ONE C-ABI handle over N devices (mm_create_multi, the handle a Go "
                         "server constructs, main.go:160): N x the per-GPU set (C3) or the whole set (C4/C5); "
                         "devices cycle over the visible GPUs (a one-GPU box: N sub-handles on device 0)")
    ap.add_argument("--multi-mode", choices=["pools", "rows"], default="pools",
                    help="with --multi-handle: MM_MULTI_POOLS (pools placed whole) or MM_MULTI_ROWS (row-sharded)")
    ap.add_argument("--front", choices=["cluster", "multi"], default=os.environ.get("NKM_BENCH_FRONT", "cluster"),
                    help="under torchrun (WORLD_SIZE > 1): 'cluster' = one process per GPU through cluster.py; "
                         "'multi' = rank 0 drives one multi-device handle over all WORLD_SIZE GPUs through the C ABI "
                         "(the other ranks only take part in the barriers)")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic file (tools/pmc_traffic.py); default the newest profiles/r0N_c<config>_traffic.json")
    a = ap.parse_args()
    if a.tickets is None:
        a.tickets = DEFAULT_TICKETS.get(a.config, 1_000_000)
    if a.traffic is None:  # the newest committed PMC pass of this config (bench.py matches kernel + tickets)
        for r in ("r06", "r05", "r04"):
            a.traffic = os.path.join(ROOT, "profiles", f"{r}_c{a.config}_traffic.json")
            if os.path.exists(a.traffic):
                break
    return a


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
    return world, rank, local, pg, backend


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


def cpu_baseline(args, searches, matched):
    """The oracle restatement of the reference's pass on this host's cores
    (the reference Go/bluge path cannot run: no Go toolchain),
    bounded to ~10-30 s of CPU: tools/cpu_baseline.py in a child process
    (this process has initialised the GPU; the child never touches it).
    C2/C3/C4: every pool's per-search time sampled at five points along its
    own pass (the earlier-matched tickets removed, the next rows searching),
    all pools concurrently, its pass = searches x the samples' trapezoid
    mean; C5: every 1000-ticket chunk pass timed whole.  `measured_full_pass`:
    whole per-pool passes of the same oracle timed offline
    (tools/make_full_golden.py), and `calibration`: the model against them
    (profiles/r04_cpu_calib_*.json)."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "tools", "cpu_baseline.py"), "--config", str(args.config),
           "--tickets", str(args.tickets), "--searches", str(searches), "--matched", str(matched)]
    if args.override:  # C5 + override: a bounded prefix of the chunk passes, extrapolated
        cmd += ["--override", "--chunks", "100"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"value": None, "unit": "tickets/s", "cores": 1, "kind": "port",
                "sample": "cpu_baseline.py failed: " + r.stderr[-300:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    out = {"value": d["value"], "unit": "tickets/s", "cores": d["cores"], "kind": "port", "sample": d["sample"],
           "all_cores": d.get("all_cores"), "algorithm": d["algorithm"], "host": d["host"]}
    name = f"c{args.config}" + ("o" if args.override else "")
    full = os.path.join(ROOT, "profiles", f"r04_cpu_full_{name}.json")
    if os.path.exists(full) and args.tickets == json.load(open(full)).get("tickets"):
        out["measured_full_pass"] = json.load(open(full))
    calib = os.path.join(ROOT, "profiles", f"r04_cpu_calib_{name}.json")
    if os.path.exists(calib) and args.tickets == json.load(open(calib)).get("tickets"):
        out["calibration"] = json.load(open(calib))["model_over_measured"]
    return out


def candidate_stats(out):
    """The pass statistics of an mm_process result (before an override's
    commit replaces it)."""
    return {"eval_ms": out.eval_ms, "eval_bytes": out.eval_bytes, "eval_launches": out.eval_launches,
            "n_batches": out.n_batches, "eval_kernel": out.eval_kernel, "pair_evals": out.pair_evals,
            "pairs_decided": out.pairs_decided}


def make_set(args, world, rank, step):
    from nakama_amd import synth
    strong = args.config in STRONG
    total = args.tickets if strong else args.tickets * world
    lo = step * total + total * rank // world
    n = total * (rank + 1) // world - total * rank // world
    if world == 1:
        return synth.TicketSet(args.config, n, first=lo)
    groups = world if args.config in (1, 2, 3) else None  # weak scaling: C3's pools times N
    return synth.TicketSet(args.config, n, first=lo, pool_groups=groups)


def numa_bind(device):
    """Binds this process to the NUMA node its GPU hangs off (the device's PCI
    numa_node, read by the library: mm_device_numa_node), like numactl
    --cpunodebind; when that is unknown, to the node the process runs on.  The
    library's host workers sit on the device's node too (mm_store.cpp
    node_cpus); this keeps the caller with them.  Called after the HIP runtime
    is up (dist_setup), before the library's first handle.  Returns the node or
    None (a one-node host)."""
    try:
        allowed = os.sched_getaffinity(0)
        nodes = []
        for nd in range(64):
            path = f"/sys/devices/system/node/node{nd}/cpulist"
            if not os.path.exists(path):
                continue
            cpus = set()
            for part in open(path).read().strip().split(","):
                if part:
                    a, _, b = part.partition("-")
                    cpus.update(range(int(a), int(b or a) + 1))
            nodes.append((nd, cpus & allowed))
        nodes = [(nd, c) for nd, c in nodes if c]
        if len(nodes) < 2:
            return None
        import nakama_amd
        want = int(nakama_amd.load_library().mm_device_numa_node(device))
        pick = next(((n, c) for n, c in nodes if n == want), None)
        if pick is None:
            import ctypes
            here = ctypes.CDLL(None).sched_getcpu()
            pick = next(((n, c) for n, c in nodes if here in c), nodes[0])
        os.sched_setaffinity(0, pick[1])
        return pick[0]
    except OSError:
        return None


def main():
    args = parse()
    world, rank, local, pg, backend = dist_setup(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # one handle over several devices: its sub-handles place themselves on
    # their devices' nodes (mm_multi.cpp), the process stays unbound
    if args.multi_handle or (world > 1 and args.front == "multi"):
        return main_multi(args, world, rank, local, pg)
    if not args.no_numa_bind:
        numa_bind(local)
    import nakama_amd
    import torch

    # SURVEY 8(d) harness pins: MaxIntervals=2, RevThreshold=0 (no wall-clock cutoff)
    from nakama_amd import synth
    mm = nakama_amd.LocalMatchmaker(max_intervals=2, device=local, rev_precision=args.config in REV, rev_threshold=0,
                                    override=(lambda groups: groups) if args.override else None)
    cm = None
    deliv = None  # pipelined delivery: the callback's counters (tools/synth.cpp SynthDelivered)
    if args.deliver and world == 1 and not args.override:
        import ctypes
        from nakama_amd import capi

        class SynthDelivered(ctypes.Structure):
            _fields_ = [(k, ctypes.c_int64) for k in ("passes", "groups", "tickets", "presences", "id_bytes", "ns")]
        deliv = SynthDelivered()
        deliv_fn = ctypes.cast(synth.lib().synth_deliver_noop, capi.DELIVER_FN)
        mm._check(mm.lib.mm_set_delivery(mm.h, deliv_fn, ctypes.byref(deliv), 2))
    deliver_ms, flush_ms = [], []
    if world > 1:
        from nakama_amd import cluster
        cm = cluster.ClusterMatchmaker(mm, pg, POOL_FIELDS[args.config],
                                       comm_device=torch.device("cuda", local) if backend == "nccl" else None,
                                       override_commit=synth.override_commit if args.override else None)
    times, matched_all, presences_all, ins_times, searched = [], [], [], [], []
    eval_ms = eval_bytes = launches = pair_evals = pairs_decided = cands = 0
    batches, kernels, unroutable = [], set(), 0
    breakdown = {"local_call_ms": [], "summary_ms": [], "merge_ms": [], "merge_wait_ms": [], "merge_comm_ms": [],
                 "merge_c_ms": []}  # rank 0's cluster-pass phases
    ov_times, step_phases = {}, {}  # --override: the step's candidate pass / override / commit
    for step in range(args.warmup + args.steps):
        ts = make_set(args, world, rank, step)
        t_ins = time.perf_counter()
        if cm is None:
            ts.insert_into(mm)  # untimed: one Insert() C-ABI call (store maintenance, index build, H2D upload)
        else:
            unroutable += len(cm.Insert(ts.ptr(), ts.n))  # untimed: route by pool, all-to-all, Insert()
        ins_dt = time.perf_counter() - t_ins
        barrier_sync(pg, local)
        t0 = time.perf_counter()
        if deliv is not None:
            out = capi.mm_matched()  # the summary: counts + statistics, the groups queued for the delivery thread
            mm._check(mm.lib.mm_process_deliver(mm.h, ctypes.byref(out)))
            t_pass = time.perf_counter()
        elif cm is None:
            out = mm.process_call()  # the C-ABI call: one whole Process() pass
            t_pass = time.perf_counter()
            n_cands = out.n_groups if out.is_candidates else 0
            cand = candidate_stats(out)  # the candidate pass ran the searches (a few scalar reads)
            if args.override and out.is_candidates:  # processCustom: override + commit, in the timed step
                out = synth.override_commit(mm, out, ov_times)
        else:
            cp = cm.Process()        # every rank's pass + the merge into the reference's group order
        barrier_sync(pg, local)
        dt = time.perf_counter() - t0
        if cm is None and args.override and step >= args.warmup:
            for k, v in (("candidate_pass_ms", 1e3 * (t_pass - t0)), ("override_ms", ov_times.get("override_ms", 0.0)),
                         ("commit_ms", ov_times.get("commit_ms", 0.0))):
                step_phases.setdefault(k, []).append(v)
        if deliv is not None:
            # untimed: wait until the no-op router has the pass (it ran behind
            # the step's end), then read what it delivered
            t_f0 = time.perf_counter()
            before_t, before_ns = deliv.tickets, deliv.ns
            mm._check(mm.lib.mm_delivery_flush(mm.h))
            if step >= args.warmup:
                flush_ms.append(1e3 * (time.perf_counter() - t_f0))
                deliver_ms.append((deliv.ns - before_ns) / 1e6)
            n_groups, matched, pres = out.n_groups, deliv.tickets - before_t, out.n_entries
            st = candidate_stats(out)
            st["candidates"] = 0
        elif cm is None:
            n_groups, matched, pres, r = mm.process_summary(out)  # untimed: counts the groups, frees them
            # the override's commit runs no search: the pass statistics are the candidate pass's
            st = dict(cand) if args.override else {
                "eval_ms": r.eval_ms, "eval_bytes": r.eval_bytes, "eval_launches": r.eval_launches,
                "n_batches": r.n_batches, "eval_kernel": r.eval_kernel, "pair_evals": r.pair_evals,
                "pairs_decided": r.pairs_decided}
            st["candidates"] = n_cands
        else:
            n_groups, matched, pres = cp.n_groups, cp.matched_tickets, cp.matched_presences
            st = cp.local_stats
            if step >= args.warmup:
                for k in breakdown:
                    breakdown[k].append(st[k])
        ts.close()
        dt_max = max_over_ranks(pg, local, dt)
        if step >= args.warmup:
            times.append(dt_max)
            ins_times.append(max_over_ranks(pg, local, ins_dt))
            matched_all.append(matched)
            presences_all.append(pres)
            # searches the pass ran: rows that were not yet selected when reached
            searched.append(n_groups + mm.ticket_count())  # C3: every leftover searched too
            eval_ms += st["eval_ms"]
            eval_bytes += st["eval_bytes"]
            launches += st["eval_launches"]
            pair_evals += st.get("pair_evals", 0)
            pairs_decided += st.get("pairs_decided", 0)
            cands += st.get("candidates", 0)
            batches.append(st["n_batches"])
            kernels.add(KERNELS.get(st["eval_kernel"], str(st["eval_kernel"])))
        # drain what is left so the next step starts from a fresh set
        mm.Remove([t.ticket for t in mm.Extract()]) if mm.ticket_count() else None
    total_t = sum(times)
    pair_evals = sum_over_ranks(pg, local, pair_evals)  # whole job (each rank counted its own pass)
    pairs_decided = sum_over_ranks(pg, local, pairs_decided)
    value = sum(matched_all) / total_t
    achieved = (eval_bytes / 1e9) / (eval_ms / 1e3) if eval_ms > 0 else 0.0
    avg_launch_ms = eval_ms / max(1, launches)
    # HBM bytes per launch from the PMC passes of the committed rocprofv3 run
    # (tools/pmc_traffic.py) — not measured in this process, labelled so
    # Only a file measured on this line's kernel, config and ticket count
    # (the PMC run's own workload) is attached; otherwise traffic is null.
    traffic, traffic_src = None, None
    if os.path.exists(args.traffic):
        try:
            tr = json.load(open(args.traffic))
            if (tr.get("kernel") in kernels and len(kernels) == 1 and tr.get("config") == args.config and
                    tr.get("tickets") == args.tickets):
                traffic, traffic_src = tr.get("bytes_per_launch"), os.path.relpath(args.traffic, ROOT)
        except Exception:
            traffic = None
    strong = args.config in STRONG
    if world == 1:
        par = "single GPU"
    elif strong:
        par = (f"pool-sharded x{world} through the cluster front: one set of {args.tickets} tickets, each rank "
               f"ingests 1/{world} and the front routes tickets to their pool's rank")
    else:
        par = (f"pool-sharded x{world} through the cluster front: one set of {world}x{args.tickets} tickets over "
               f"{world}x the config's pools, each rank ingests {args.tickets} and the front routes tickets to "
               f"their pool's rank")
    out = {
        "metric": "tickets matched/sec + Process() interval p50 latency at 1M active tickets",
        "value": value,
        "unit": "tickets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * total_t / args.steps,
        "p50_ms": 1e3 * statistics.median(times),
        "step_ms": [round(1e3 * t, 3) for t in times],  # every timed step (max over ranks), in order
        "presences_per_s": sum(presences_all) / total_t,
        # (row, candidate) predicate evaluations the device issued: one per
        # candidate scanned by a search (a shared search decides all its rows
        # at once; the hashed scan tests each candidate against the one
        # signature its values select), per second of the timed steps
        "pair_evals_per_s": pair_evals / total_t,
        # (row, candidate) pairs decided: over the rows that searched, the
        # candidates of their search's source — the posting list of the
        # query's most selective required term, which bluge's conjunction
        # searcher walks (C3: the row's region list, 2 modes x 125k = 250k,
        # not its 125k pool) — what the reference's per-row bluge search
        # evaluates (BASELINE.md GPU-side reporting), summed over ranks.
        # Check: pairs_decided_per_s x ms_per_step / 1e3 = searches_per_pass x
        # that source length.
        "pairs_decided_per_s": pairs_decided / total_t,
        "searches_per_pass": statistics.median(searched) if searched else None,
        # the host-to-HBM hand-over: the Insert() call that precedes each pass
        # (not part of value: inputs are resident when the timed region starts)
        "insert_ms": 1e3 * statistics.median(ins_times),
        "with_insert_tickets_per_s": sum(matched_all) / (total_t + sum(ins_times)),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "int64/f64",
        "data": "synthetic",
        "config": {"workload": WORKLOADS.get(args.config, str(args.config)) +
                               (" + MatchmakerOverride (processCustom candidates, native first-disjoint override, "
                                "mm_process_commit)" if args.override else
                                " (processDefault: no override registered)" if args.config in REV else ""),
                   ("tickets_total" if strong else "tickets_per_gpu"): args.tickets,
                   "max_intervals": 2, "parallelism": par, "unroutable": unroutable,
                   "matched_per_step": sum(matched_all) / args.steps, "batches_per_pass_rank0": batches,
                   "candidates_per_pass": (cands / args.steps) if args.override else None,
                   "cluster_phases_ms_rank0": ({k: statistics.median(v) for k, v in breakdown.items()}
                                               if cm is not None else None),
                   # --override: medians of the step's parts (the override is the bench's native
                   # first-disjoint stand-in for the user's MatchmakerOverride, runtime.go:212)
                   "override_step_ms": ({k: statistics.median(v) for k, v in step_phases.items()}
                                        if step_phases else None),
                   # the default (--no-deliver off): the timed step ends when mm_process_deliver returns (the pass done, its
                   # result queued); the no-op router's callback runs on the delivery thread behind it
                   "delivery": ({"mode": "pipelined (mm_process_deliver, depth 2)",
                                 "callback_ms_p50": statistics.median(deliver_ms),
                                 "flush_wait_ms_p50": statistics.median(flush_ms),
                                 "tickets_delivered_per_step": sum(matched_all) / args.steps}
                                if deliver_ms else None)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "+".join(sorted(kernels)), "launches": launches, "avg_launch_ms": avg_launch_ms,
                     "bytes_per_launch": eval_bytes / max(1, launches), "rank": 0},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config in (2, 3, 4, 5):
        out["cpu_baseline"] = cpu_baseline(args, int(statistics.median(searched)), int(statistics.median(matched_all)))
    else:
        out["cpu_baseline"] = None
    mm.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.barrier()
        pg.destroy_process_group()


def main_multi(args, world, rank, local, pg):
    """ONE matchmaker handle over N devices in this process, through the C ABI
    (mm_create_multi, include/nakama_cluster.h) — what a Go server
    constructs (main.go:160) with the INTEGRATION.md shim.  Under torchrun
    (--front multi) rank 0 drives all WORLD_SIZE GPUs and the other ranks
    only join the barriers; alone (--multi-handle N) the process drives N
    sub-handles over the visible GPUs.  Same step as main(): insert a fresh set
    (untimed: routed by pool inside the library), one timed Process()."""
    import torch

    import nakama_amd
    from nakama_amd import capi, synth
    n_sub = args.multi_handle or world
    visible = max(1, torch.cuda.device_count())
    devs = [i % visible for i in range(n_sub)]
    strong = args.config in STRONG
    total = args.tickets if strong else args.tickets * n_sub
    mm = None
    if rank == 0:
        if world > 1:
            os.environ["LOCAL_WORLD_SIZE"] = "1"  # the other ranks sit idle: the sub-handles share all host cores
        mode = capi.MM_MULTI_ROWS if args.multi_mode == "rows" else capi.MM_MULTI_POOLS
        mm = nakama_amd.LocalMatchmaker(max_intervals=2, rev_precision=args.config in REV, rev_threshold=0,
                                        override=(lambda groups: groups) if args.override else None,
                                        multi=dict(devices=devs, mode=mode, pool_fields=list(POOL_FIELDS[args.config])))
    times, matched_all, presences_all, ins_times = [], [], [], []
    eval_ms = eval_bytes = launches = pair_evals = pairs_decided = cands = 0
    batches, kernels = [], set()
    for step in range(args.warmup + args.steps):
        ins_dt = dt = 0.0
        if rank == 0:
            groups = n_sub if (args.config in (1, 2, 3) and n_sub > 1) else None
            ts = synth.TicketSet(args.config, total, first=step * total, pool_groups=groups)
            t_ins = time.perf_counter()
            ts.insert_into(mm)  # untimed: routed to the sub-handles by pool (or replicated: rows)
            ins_dt = time.perf_counter() - t_ins
        barrier_sync(pg, local)
        t0 = time.perf_counter()
        if rank == 0:
            out = mm.process_call()
            n_cands = out.n_groups if out.is_candidates else 0
            cand = candidate_stats(out)
            if args.override and out.is_candidates:
                out = synth.override_commit(mm, out)
            for d in sorted(set(devs)):
                torch.cuda.synchronize(d)
        barrier_sync(pg, local)
        dt = time.perf_counter() - t0
        if rank == 0:
            n_groups, matched, pres, r = mm.process_summary(out)
            ts.close()
            if step >= args.warmup:
                times.append(dt)
                ins_times.append(ins_dt)
                matched_all.append(matched)
                presences_all.append(pres)
                st = cand if args.override else candidate_stats(r)
                eval_ms += st["eval_ms"]
                eval_bytes += st["eval_bytes"]
                launches += st["eval_launches"]
                pair_evals += st["pair_evals"]
                pairs_decided += st["pairs_decided"]
                cands += n_cands
                batches.append(st["n_batches"])
                kernels.add(KERNELS.get(st["eval_kernel"], str(st["eval_kernel"])))
            mm.Remove([t.ticket for t in mm.Extract()]) if mm.ticket_count() else None
    if rank == 0:
        total_t = sum(times)
        achieved = (eval_bytes / 1e9) / (eval_ms / 1e3) if eval_ms > 0 else 0.0
        n_dev = len(set(devs))
        out = {
            "metric": "tickets matched/sec + Process() interval p50 latency at 1M active tickets",
            "value": sum(matched_all) / total_t,
            "unit": "tickets/s",
            "n_gpus": n_dev,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * total_t / args.steps,
            "p50_ms": 1e3 * statistics.median(times),
        "step_ms": [round(1e3 * t, 3) for t in times],  # every timed step (max over ranks), in order
            "presences_per_s": sum(presences_all) / total_t,
            "pair_evals_per_s": pair_evals / total_t,
            "pairs_decided_per_s": pairs_decided / total_t,
            "insert_ms": 1e3 * statistics.median(ins_times),
            "with_insert_tickets_per_s": sum(matched_all) / (total_t + sum(ins_times)),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic",
            "config": {"workload": WORKLOADS.get(args.config, str(args.config)) +
                                   (" + MatchmakerOverride" if args.override else ""),
                       ("tickets_total" if strong else "tickets_per_gpu"): args.tickets,
                       "max_intervals": 2,
                       "parallelism": (f"one C-ABI handle over {n_sub} sub-handles (mm_create_multi, "
                                       f"{'MM_MULTI_ROWS' if args.multi_mode == 'rows' else 'MM_MULTI_POOLS'}) on "
                                       f"devices {devs}" + (" (one GPU: the sub-handles share it)" if n_dev < n_sub
                                                            else "")),
                       "matched_per_step": sum(matched_all) / args.steps, "batches_per_pass": batches,
                       "candidates_per_pass": (cands / args.steps) if args.override else None},
            # the sub-handles' launches run concurrently: eval time is the slowest device's
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "traffic_source": None,
                         "kernel": "+".join(sorted(kernels)), "launches": launches,
                         "avg_launch_ms": eval_ms / max(1, launches), "bytes_per_launch": eval_bytes / max(1, launches),
                         "note": "eval bytes of the sub-handles on the dominant kernel / the slowest sub-handle's "
                                 "event time"},
            "cpu_baseline": None,
        }
        mm.close()
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.barrier()
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
