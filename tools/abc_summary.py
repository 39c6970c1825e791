#!/usr/bin/env python3
"""One line per bench run of gpurun_out/abc.jsonl (tools/gpu_ab_configs.sh)."""
import json
import sys

for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abc.jsonl"):
    d = json.loads(l)
    r = d["roofline"]
    print(d["tree"][:6].ljust(6), d["args"][:28].ljust(28), "M/s %7.2f" % (d["value"] / 1e6), "p50 %7.2f" % d["p50_ms"],
          r["kernel"][:22].ljust(22), "us %8.1f" % (r["avg_launch_ms"] * 1e3), "frac %.3f" % r["frac"],
          "B/l %.3g" % r["bytes_per_launch"], d["config"]["batches_per_pass_rank0"])
