"""A small, repeatable driver for profiling the check kernels on a saved snapshot: the first
run (--save DIR) generates the workload, builds the snapshot and saves it with the requests;
later runs (--load DIR) start from the file (seconds instead of minutes), so rocprofv3
counter passes over the same launches stay cheap.  Runs `--steps` HBM-resident batches.

    python tools/label_probe.py --save /tmp/c2            # config #2, once
    rocprofv3 --pmc ... -- python3 tools/label_probe.py --load /tmp/c2
"""
import argparse
import json
import os
import sys
import time

import torch  # noqa: F401
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd import check  # noqa: E402
from keto_amd.snapshot import Snapshot  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--save", default=None)
    p.add_argument("--load", default=None)
    p.add_argument("--workload", choices=["rbac", "folders", "social"], default="rbac")
    p.add_argument("--tuples", type=int, default=50_000_000)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--host", action="store_true", help="also time host-to-host batches (pinned requests)")
    a = p.parse_args()
    t0 = time.time()
    if a.load:
        meta = json.load(open(os.path.join(a.load, "meta.json")))
        snap = Snapshot.load(os.path.join(a.load, "graph.snap"), [tuple(x) for x in meta["namespaces"]])
        z = np.load(os.path.join(a.load, "requests.npz"))
        roots, targets = z["roots"], z["targets"]
    else:
        from tools.bench_scale import make
        w = make(a.workload, a.tuples, 1_000_000)
        snap = Snapshot.from_columns(w.namespaces, w.columns)
        roots, targets = w.resolve(snap)
        if a.save:
            os.makedirs(a.save, exist_ok=True)
            snap.save(os.path.join(a.save, "graph.snap"))
            np.savez(os.path.join(a.save, "requests.npz"), roots=roots, targets=targets)
            json.dump({"namespaces": [list(x) for x in w.namespaces]}, open(os.path.join(a.save, "meta.json"), "w"))
    t_load = time.time() - t0
    t0 = time.time()
    eng = check.Engine(snap)
    t_eng = time.time() - t0
    q = eng.upload(roots, targets)
    for _ in range(2):
        q.run()
    t0 = time.perf_counter()
    calls, gpu = [], []
    for _ in range(a.steps):
        c0 = time.perf_counter()
        q.run()
        calls.append(time.perf_counter() - c0)
        gpu.append(eng.last_stats()["ms_total"])
    dt = (time.perf_counter() - t0) / a.steps
    lean = eng.last_stats()
    eng.set_events(True)  # the first stage's own time (events between the kernels)
    ms = []
    for _ in range(a.steps):
        q.run()
        ms.append(eng.last_stats()["main_ms"])
    eng.set_events(False)
    st = eng.last_stats()
    out = {"load_s": round(t_load, 1), "engine_s": round(t_eng, 2), "plan": st["plan"],
           "hbm_checks_per_s": round(len(roots) / dt, 1), "main_ms_median": round(float(np.median(ms)), 4),
           "main_bytes": st["main_bytes"], "label_build_ms": round(st["label_build_ms"], 1),
           "allowed": int(q.download().sum()),
           # per call: host wall time vs the GPU span between the call's first and last event
           "call_us_median": round(float(np.median(calls)) * 1e6, 1),
           "gpu_span_us_median": round(float(np.median(gpu)) * 1e3, 1),
           "full_requests": st["full_requests"], "rest_requests": st["rest_requests"],
           "lean_full_requests": lean["full_requests"],
           "heads": f'{st["label_s_head"]},{st["label_p_head"]}', "label_bytes": st["label_bytes"]}
    if a.host:
        pr, pt = check.pinned(roots), check.pinned(targets)
        out_b = check.PinnedBuffer((len(roots) + 63) // 64, np.uint64)
        for _ in range(3):
            eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, len(roots), out_b.array.ctypes.data)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, len(roots), out_b.array.ctypes.data)
        out["host_checks_per_s"] = round(len(roots) * a.steps / (time.perf_counter() - t0), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
