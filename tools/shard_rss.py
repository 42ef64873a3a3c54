"""Per-rank host memory of the partition-aware loader against world size (CPU, gloo).

    python tools/shard_rss.py --scale 0.01 --worlds 1,2,4,8 --out profiles/r02/shard_rss.json

For each world size, `world` processes (gloo over 127.0.0.1) stream the same config #5
row stream (synth.config5 at --scale x 5B tuples) through Shard.load — the loader and id
exchange of the partitioned mode, no device involved — and report per rank: the loader's
host arrays (ketogpu_shard_stats.host_bytes), peak RSS before and after the load, the
owned nodes/edges and the load time.  The loader's arrays and the RSS growth should fall
as 1/world (every rank still reads the whole stream, but keeps only what it owns).
"""
import argparse
import json
import os
import resource
import socket
import sys
import time

import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


def worker(rank, world, port, scale, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from keto_amd import synth
    from keto_amd.partition import Shard
    sizes = dict(users=max(1000, int(500_000_000 * scale)), groups=max(100, int(10_000_000 * scale)),
                 docs=max(100, int(200_000_000 * scale)), tuples=max(10_000, int(5_000_000_000 * scale)))
    w = synth.config5(**sizes, checks=1000)
    r0 = rss_gb()
    t0 = time.time()
    sh = Shard.load(w.namespaces, lambda: w.batches(1 << 20))
    dt = time.time() - t0
    st = sh.stats()
    q.put({"rank": rank, "rss_before_gb": round(r0, 3), "peak_rss_gb": round(rss_gb(), 3),
           "rss_growth_gb": round(rss_gb() - r0, 3), "loader_array_gb": round(st["host_bytes"] / 1e9, 3),
           "rows_streamed": st["rows"], "owned_nodes": st["owned_nodes"],
           "owned_interior": st["owned_interior"], "forward_edges": st["forward_edges"],
           "reverse_edges": st["reverse_edges"], "load_s": round(dt, 1)})
    sh.close()
    dist.barrier()
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.004)
    ap.add_argument("--worlds", default="1,2,4")
    ap.add_argument("--out", default="-", help="JSON file (default stdout; gloo logs to stdout too)")
    a = ap.parse_args()
    out = {"workload": f"config5 x{a.scale} ({int(5e9 * a.scale)} tuples)", "backend": "gloo (CPU)", "runs": []}
    ctx = mp.get_context("spawn")
    for world in [int(x) for x in a.worlds.split(",")]:
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=worker, args=(r, world, port, a.scale, q)) for r in range(world)]
        for p in procs:
            p.start()
        ranks = sorted((q.get() for _ in range(world)), key=lambda d: d["rank"])
        for p in procs:
            p.join()
            if p.exitcode:
                raise SystemExit(f"rank exited with {p.exitcode}")
        out["runs"].append({"world": world, "ranks": ranks,
                            "max_loader_array_gb": max(r["loader_array_gb"] for r in ranks),
                            "max_rss_growth_gb": max(r["rss_growth_gb"] for r in ranks)})
        print(f"[shard_rss] world {world}: loader arrays {[r['loader_array_gb'] for r in ranks]} GB, "
              f"RSS growth {[r['rss_growth_gb'] for r in ranks]} GB", file=sys.stderr, flush=True)
    base = out["runs"][0]
    for r in out["runs"]:
        r["loader_array_ratio_vs_world1"] = round(r["max_loader_array_gb"] / base["max_loader_array_gb"], 3)
        r["rss_growth_ratio_vs_world1"] = round(r["max_rss_growth_gb"] / max(base["max_rss_growth_gb"], 1e-9), 3)
    text = json.dumps(out, indent=1)
    if a.out == "-":
        print(text)
    else:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
