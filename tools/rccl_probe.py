"""Probe of the row-sharded RCCL transport at world 1 (one process): prints
each step so a hang names its step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
torch.cuda.set_device(0)
print("init pg", flush=True)
world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
dist.init_process_group(os.environ.get("PROBE_BACKEND", "gloo"), rank=rank, world_size=world)
import nakama_amd  # noqa: E402
from nakama_amd import capi, cluster, synth  # noqa: E402

mm = nakama_amd.LocalMatchmaker(max_intervals=2)
print("row shard init", flush=True)
rm = cluster.RowShardedMatchmaker(mm, dist, transport="rccl")
print("insert", flush=True)
ts = synth.TicketSet(9, 2000 // world, first=rank * (2000 // world))
rm.Insert(ts.ptr(), ts.n)
print("process", flush=True)
t0 = time.time()
r = rm.Process()
print("groups", len(r.groups), "batches", r.n_batches, f"{time.time() - t0:.3f}s", flush=True)
mm.close()
dist.destroy_process_group()
print("ok", flush=True)
