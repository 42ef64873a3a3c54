"""How many of plan label's requests would the first stage answer with more landmarks kept
as mask bits?  A CPU study over the host build of the label heads (labels.cpp build_labels,
`Snapshot.label_index`): for a sample of requests it decodes P(root) and S(target), then
replays the first stage's decision (masks share a bit, or the first head - 4 entries of the
two lists meet; else a list longer than its head sends the request to the dense pass) with
the landmarks of rank < 64 + M moved from the lists into the masks.

    python tools/label_mask_study.py --workload folders --tuples 5000000 --sample 20000

Prints one JSON line per M: the dense-pass share and the mean list lengths.  (Rank order is
the labeller's centrality order, so the moved landmarks are the lists' first entries.)  The
last line drops the raw entries (node ids, not landmarks) from both lists and answers the
one-edge case r in rev(t) by a separate test instead.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd.snapshot import Snapshot  # noqa: E402
from tools.bench_scale import make  # noqa: E402

HEAD_FIXED = 4


def decode(arr, h, x):
    """the list and 64-bit mask of node x (head words h)"""
    head = arr[x * h:(x + 1) * h]
    c = int(head[0])
    mask = int(head[2]) | int(head[3]) << 32
    if c == 0xFFFFFFFF:
        return None, 0
    if c > h - HEAD_FIXED:
        o = int(head[1]) * 16
        return arr[o:o + c].astype(np.int64), mask
    return head[HEAD_FIXED:HEAD_FIXED + c].astype(np.int64), mask


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["rbac", "folders", "social"], default="folders")
    p.add_argument("--tuples", type=int, default=5_000_000)
    p.add_argument("--sample", type=int, default=20000)
    p.add_argument("--extra", default="0,64,192,448,960", help="landmarks moved into the masks beyond the first 64")
    p.add_argument("--inline", default="", help="inline entries per head to replay instead of the built heads' "
                                                "(e.g. 60,28: 64-word S heads, 32-word P heads)")
    a = p.parse_args()
    w = make(a.workload, a.tuples, a.sample)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    li = snap.label_index(0, 0)
    S, P, hs, hp = li["S"], li["P"], li["s_head_words"], li["p_head_words"]
    ni = int(snap.stats()["num_interior"])
    cases = []
    for r, t in zip(roots.tolist(), targets.tolist()):
        if r == 0xFFFFFFFF or t == 0xFFFFFFFF:
            continue
        pl, pm = decode(P, hp, r)
        sl, sm = decode(S, hs, t)
        if pl is None or sl is None:
            continue
        cases.append((pl, pm, sl, sm))
    cap_s, cap_p = (int(x) for x in a.inline.split(",")) if a.inline else (hs - HEAD_FIXED, hp - HEAD_FIXED)
    for m, raw in [(int(x), True) for x in a.extra.split(",")] + [(0, False), (448, False)]:
        bound = 64 + m
        dense = answered = 0
        lp = ls = 0
        for pl, pm, sl, sm in cases:
            if not raw:
                # raw entries (node ids >= ni) serve only the one-edge test r in rev(t): P's
                # one raw entry is r itself — answered by a separate edge test, the lists
                # keep their landmarks
                if (pl[pl >= ni][:, None] == sl[sl >= ni][None, :]).any():
                    answered += 1
                    lp += int((pl < ni).sum())
                    ls += int((sl < ni).sum())
                    continue
                pl, sl = pl[pl < ni], sl[sl < ni]
            # landmarks below `bound` leave the lists for the masks (raw ids >= ni stay)
            pk = pl[(pl >= bound) | (pl >= ni)]
            sk = sl[(sl >= bound) | (sl >= ni)]
            pmk = set(pl[(pl < bound) & (pl < ni)].tolist())
            smk = set(sl[(sl < bound) & (sl < ni)].tolist())
            lp += len(pk)
            ls += len(sk)
            hit = (pm & sm) != 0 or bool(pmk & smk)
            if not hit:
                hit = bool(np.intersect1d(pk[:cap_p], sk[:cap_s]).size)
            if hit:
                answered += 1
            elif len(pk) > cap_p or len(sk) > cap_s:
                dense += 1
            else:
                answered += 1
        n = max(len(cases), 1)
        print(json.dumps({"workload": a.workload, "tuples": a.tuples, "heads": [hs, hp], "inline": [cap_s, cap_p],
                          "mask_bits": bound,
                          "raw_entries_in_lists": raw,
                          "requests": len(cases), "dense_pass_share": round(dense / n, 4),
                          "first_stage_share": round(answered / n, 4), "mean_p_entries": round(lp / n, 2),
                          "mean_s_entries": round(ls / n, 2)}), flush=True)


if __name__ == "__main__":
    main()
