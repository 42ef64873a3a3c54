"""Which requests does plan label's dense pass get on the config #2 shape, and why?  A CPU
replay of the first stage's decision (device_engine.hip label_unit; tests/test_core_index.py
first_stage) over the host build of the heads at 32/32 words: for every request the heads do
not settle it counts whether P or S overflows and, when S is whole and P is not, how many of
S's landmarks lie above P's last inline entry (the ones the prefix rule cannot rule out).

    python tools/label_dense_study.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd.snapshot import Snapshot
from tools.bench_scale import make
from tools.label_format_study import decode, mask_ranks
w = make('rbac', 5_000_000, 20000)
snap = Snapshot.from_columns(w.namespaces, w.columns)
roots, targets = w.resolve(snap)
li = snap.label_index(32, 32)
S, P, hs, hp = li["S"], li["P"], li["s_head_words"], li["p_head_words"]
ni = int(snap.stats()["num_interior"])
cs = cp = 28
dense = 0; und_hist = {}; p_over = 0; s_over = 0; both = 0
for r, t in zip(roots.tolist(), targets.tolist()):
    if r == 0xFFFFFFFF or t == 0xFFFFFFFF: continue
    pl, pm = decode(P, hp, r); sl, sm = decode(S, hs, t)
    if pm & sm: continue
    slm = sl[sl < ni]; raw = sl[sl >= ni]
    s_in = sl[:cs]; p_in = pl[:cp]
    if np.intersect1d(s_in[s_in < ni], p_in).size: continue
    if r >= ni and (s_in == r).any(): continue
    s_whole = len(sl) <= cs or s_in[-1] >= ni
    p_whole = len(pl) <= cp
    es = (s_in < ni).sum(); ep = min(len(pl), cp)
    s_last = s_in[es-1] if es else 0; p_last = p_in[ep-1] if ep else 0
    lm = es == 0 or len(pl) == 0 or (s_whole and (p_whole or s_last <= p_last)) or (p_whole and p_last <= s_last)
    rawd = r < ni or len(sl) <= cs or r <= s_in[-1]
    if lm and rawd: continue
    dense += 1
    p_over += not p_whole; s_over += not s_whole; both += (not p_whole) and (not s_whole)
    if s_whole and not p_whole:
        k = int((slm > p_last).sum()); und_hist[k] = und_hist.get(k, 0) + 1
n = len(roots)
print("dense", dense/n, "p_over", p_over, "s_over", s_over, "both", both)
print("S-whole & P-partial: S landmarks above P's last inline:", sorted(und_hist.items())[:12])
