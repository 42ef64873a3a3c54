"""A/B the LDS unit plans on config #2 in ONE process (same graph, same requests):
KETOGPU_UNITS = bidi[:hlog] | v2 | w4 | w8 | w16 | b16, plus the global path.  Prints ms per 1M-request
run (median of interleaved rounds) and checks every plan returns identical bits."""
import os
import sys
import time

import torch  # noqa: F401  (same HIP runtime as bench.py)
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd import check, synth  # noqa: E402
from keto_amd.snapshot import Snapshot  # noqa: E402

small = "--small" in sys.argv
scale = 100 if small else 1
workload = next((a.split("=")[1] for a in sys.argv if a.startswith("--workload=")), "rbac")
if workload == "folders":  # config #3 shape at 5M tuples
    w = synth.folders(users=100_000, groups=1_000, folders=200_000, tuples=5_000_000, checks=1_000_000)
elif workload == "social":  # config #4 shape at 5M tuples
    w = synth.social(users=500_000, groups=50_000, tuples=5_000_000, checks=1_000_000)
else:
    w = synth.rbac(users=10_000_000 // scale, groups=100_000 // scale, docs=2_000_000 // scale,
                   tuples=50_000_000 // scale, checks=1_000_000)
snap = Snapshot.from_columns(w.namespaces, w.columns)
roots, targets = w.resolve(snap)
plans = [p for p in sys.argv[1:] if not p.startswith("--")] or ["w4", "w8", "w16", "b16", "global"]
engines, queries = {}, {}
for p in plans:
    if p == "global":
        os.environ["KETOGPU_PATH"] = "global"
    else:  # plan[:first[/cascade]][@both,seed], e.g. bidi:9,64,128,7/q,s@12,32
        os.environ.pop("KETOGPU_PATH", None)
        os.environ.pop("KETOGPU_BIDI", None)
        os.environ.pop("KETOGPU_CASCADE", None)
        os.environ.pop("KETOGPU_BIDI_TUNE", None)
        spec, _, tune = p.partition("@")  # bidi[:first[/wide]][@both,seed]
        if tune:
            os.environ["KETOGPU_BIDI_TUNE"] = tune
        os.environ["KETOGPU_UNITS"] = spec.split(":")[0]
        if ":" in spec:
            first, _, wide = spec.split(":")[1].partition("/")
            if first:
                os.environ["KETOGPU_BIDI"] = first
            if wide:
                os.environ["KETOGPU_CASCADE"] = wide
    engines[p] = check.Engine(snap, state_budget_bytes=16 << 30)
    queries[p] = engines[p].upload(roots, targets)
ref = None
times = {p: [] for p in plans}
for rnd in range(5):
    for p in plans:
        q = queries[p]
        t0 = time.perf_counter()
        q.run()
        times[p].append(time.perf_counter() - t0)
        if rnd == 0:
            got = q.download()
            if ref is None:
                ref = got
            assert np.array_equal(got, ref), f"plan {p} differs"
for p in plans:
    st = engines[p].last_stats()
    print(f"{p:7s} median {np.median(times[p]) * 1e3:8.3f} ms  min {min(times[p]) * 1e3:8.3f}  "
          f"unit {st['ms_unit']:.3f} ms push {st['ms_push']:.3f} spilled_units {st['spilled_units']} "
          f"spilled_req {st['spilled_requests']}", flush=True)
