"""A/B of plan label's head sizes (KETOGPU_LABEL_HEADS) on one snapshot: every variant's
engine is timed host to host (pinned requests) and HBM-resident, its answers diffed
against the first variant's, on the config #2 workload (or --workload).

    python tools/label_ab.py --heads 0,0 16,16 32,16
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
from tools.bench_scale import make  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["rbac", "folders", "social"], default="rbac")
    p.add_argument("--tuples", type=int, default=50_000_000)
    p.add_argument("--users", type=int, default=None)
    p.add_argument("--groups", type=int, default=None)
    p.add_argument("--heads", nargs="+", default=["0,0"])
    p.add_argument("--env", nargs="*", default=[], help="extra KEY=VALUE per run (applied to every variant)")
    p.add_argument("--steps", type=int, default=20)
    a = p.parse_args()
    w = make(a.workload, a.tuples, 1_000_000, a.users, a.groups)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    pos = w.chk_pos.astype(bool)
    del w
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    n = len(roots)
    pr, pt = check.pinned(roots), check.pinned(targets)
    out = check.PinnedBuffer((n + 63) // 64, np.uint64)
    ref = None
    for h in a.heads:
        os.environ["KETOGPU_LABEL_HEADS"] = h
        t0 = time.time()
        eng = check.Engine(snap)
        t_eng = time.time() - t0
        step = lambda: eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, n, out.array.ctypes.data)
        for _ in range(3):
            step()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        dt = (time.perf_counter() - t0) / a.steps
        got = check.unpack_bits(out.array.copy(), n)
        eng.set_events(True)
        step()
        st_h = eng.last_stats()
        eng.set_events(False)
        q = eng.upload(roots, targets)
        for _ in range(3):
            q.run()
        t0 = time.perf_counter()
        ms = []
        for _ in range(a.steps):
            q.run()
            ms.append(eng.last_stats()["main_ms"])
        dt_res = (time.perf_counter() - t0) / a.steps
        st = eng.last_stats()
        cs = [q] + [eng.upload(roots, targets) for _ in range(1)]  # pipelined: no host wait per call
        for qq in cs[1:]:                                         # (ketogpu_queries_run_async), two
            qq.run()                                              # copies of the batch over two streams
        t0 = time.perf_counter()
        for k in range(a.steps):
            cs[k % 2].run(pipelined=True)
        eng.wait()
        dt_pipe = (time.perf_counter() - t0) / a.steps
        for qq in cs:
            assert np.array_equal(qq.download(), ref if ref is not None else got)
        for qq in cs[1:]:
            qq.close()
        eng.set_events(True)  # the first stage's own time and the dense pass's requests
        q.run()
        st_ev = eng.last_stats()
        eng.set_events(False)
        if ref is None:
            ref = got
        print(json.dumps({"heads": h, "s_head": st["label_s_head"], "p_head": st["label_p_head"],
                          "plan": st["plan"], "host_checks_per_s": round(n / dt, 1), "host_kernel_ms": round(st_h["main_ms"], 4),
                          "hbm_checks_per_s": round(n / dt_res, 1), "pipelined_checks_per_s": round(n / dt_pipe, 1),
                          "first_stage_ms": round(st_ev["main_ms"], 4), "dense_requests": st_ev["full_requests"],
                          "rest_requests": st_ev["rest_requests"], "after_first_stage_ms": round(st_ev["rest_ms"], 4),
                          "main_bytes": st["main_bytes"], "label_bytes": st["label_bytes"],
                          "engine_s": round(t_eng, 2), "mismatches_vs_first": int((got != ref).sum()),
                          "positives_denied": int((pos & ~got.astype(bool)).sum())}), flush=True)
        del q, eng


if __name__ == "__main__":
    main()
