"""Host cost of a pipelined resident call (ketogpu_queries_run_async) on the config #2 graph:
the time to ENQUEUE K calls (before waiting) against the time until they are done, and the
ctypes round trip of a trivial entry point.  If enqueueing takes as long as the GPU work, the
pipelined rate is bound by the host, not by the kernels.

    python tools/host_enqueue_probe.py [--tuples 50000000] [--calls 200]
"""
import argparse
import json
import os
import sys
import time

import torch  # noqa: F401
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd import _lib as L  # noqa: E402
from keto_amd import check  # noqa: E402
from keto_amd.snapshot import Snapshot  # noqa: E402
from tools.bench_scale import make  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="rbac")
    p.add_argument("--tuples", type=int, default=50_000_000)
    p.add_argument("--calls", type=int, default=200)
    a = p.parse_args()
    w = make(a.workload, a.tuples, 1_000_000)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    eng = check.Engine(snap)
    q, q2 = eng.upload(roots, targets), eng.upload(roots, targets)
    for qq in (q, q2):
        qq.run()
    lib = L.lib()
    t0 = time.perf_counter()
    for _ in range(1000):
        lib.ketogpu_abi_version()
    ctypes_us = (time.perf_counter() - t0) * 1e3
    out = {"ctypes_trivial_call_us": round(ctypes_us, 3)}
    for mode in ("pipelined", "sync"):
        eng.wait()
        t0 = time.perf_counter()
        for k in range(a.calls):
            (q if k % 2 == 0 else q2).run(pipelined=(mode == "pipelined"))
        t_enq = time.perf_counter() - t0
        eng.wait()
        t_all = time.perf_counter() - t0
        out[mode] = {"enqueue_us_per_call": round(t_enq / a.calls * 1e6, 2),
                     "total_us_per_call": round(t_all / a.calls * 1e6, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
