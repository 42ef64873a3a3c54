"""Host build of plan label's 2-hop labels and heads on a generated graph (CPU only): the
build time, the label sizes and the head arrays' shape, without a GPU.

    python tools/label_build.py --workload rbac --tuples 50000000
    python tools/label_build.py --workload social --tuples 100000000 --groups 10000000
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_scale import make  # noqa: E402
from keto_amd.snapshot import Snapshot  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["rbac", "folders", "social"], default="rbac")
    p.add_argument("--tuples", type=int, default=50_000_000)
    p.add_argument("--users", type=int, default=None)
    p.add_argument("--groups", type=int, default=None)
    a = p.parse_args()
    t0 = time.time()
    w = make(a.workload, a.tuples, 1000, a.users, a.groups)
    t_gen = time.time() - t0
    t0 = time.time()
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    t_snap = time.time() - t0
    del w
    st = snap.stats()
    t0 = time.time()
    li = snap.label_index()
    t_lab = time.time() - t0
    out = {k: v for k, v in li.items() if k not in ("S", "P")}
    out.update(workload=a.workload, tuples=a.tuples, generate_s=round(t_gen, 1), snapshot_s=round(t_snap, 1),
               label_s=round(t_lab, 2), bytes=4 * (len(li["S"]) + len(li["P"])),
               nodes=st["num_nodes"], interior=st["num_interior"], expandable=st["num_expandable"])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
