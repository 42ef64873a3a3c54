"""Which head format should plan label use?  A CPU replay of the first stage's decision for
the landmark-only format (labels.hpp, format 2) over the host build of the 2-hop labels.

For a sample of requests (r, t) it decodes the full landmark lists Lp = P(r), Ls = S(t) and
the raw entries of S(t) (non-interior members of rev(t)) from `Snapshot.label_index`, then,
per candidate format (S head words HS, P head words HP, mask bits MB), replays:

  * landmarks of rank < MB are mask bits, the others list entries; a head holds
    HS - 4 - MB/32 inline entries (header: landmark count, raw count, overflow start, spare;
    then the mask words): the landmarks ascending, then the raw entries ascending;
  * hit: the masks share a bit, the inline landmark prefixes meet, or (r not interior) r is
    among the inline raw entries;
  * otherwise the request is decided when the landmark test is decided — both landmark
    lists whole in their heads, or one whole with its largest entry <= the other's last
    inline entry (the prefix rule: a common landmark would be in both prefixes) — and the
    raw test is decided (r interior, no raw entries, all raw entries inline, or r <= the
    last inline raw entry); else it goes to the dense pass.

Prints one JSON line per format: dense-pass share, 128-byte lines read per request by the
first stage (a head of 64 words = 2 lines, <= 32 words = 1), and the mean list lengths.

    python tools/label_format_study.py --workload folders --tuples 5000000 --sample 20000
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from keto_amd.snapshot import Snapshot  # noqa: E402
from tools.bench_scale import make  # noqa: E402

HEAD_FIXED = 4  # format 1 (the built heads): count, overflow start, mask lo, mask hi


def decode(arr, h, x):
    """format-1 head of node x -> (entries, 64-bit mask) or (None, 0) without a label"""
    head = arr[x * h:(x + 1) * h]
    c = int(head[0])
    if c == 0xFFFFFFFF:
        return None, 0
    mask = int(head[2]) | int(head[3]) << 32
    if c > h - HEAD_FIXED:
        o = int(head[1]) * 16
        return arr[o:o + c].astype(np.int64), mask
    return head[HEAD_FIXED:HEAD_FIXED + c].astype(np.int64), mask


def mask_ranks(mask):
    return np.array([k for k in range(64) if (mask >> k) & 1], dtype=np.int64)


def replay(cases, ni, hs, hp, mb, prefix_rule=True):
    cap_s, cap_p = hs - 4 - mb // 32, hp - 4 - mb // 32
    dense = 0
    ls = lp = lr = 0
    for lmp, lms, raw, r in cases:
        mp, mpl = lmp[lmp < mb], lmp[lmp >= mb]
        ms, msl = lms[lms < mb], lms[lms >= mb]
        ls += len(msl)
        lp += len(mpl)
        lr += len(raw)
        if np.intersect1d(mp, ms, assume_unique=True).size:
            continue
        s_in = np.concatenate([msl, raw])[:cap_s]  # the S head's inline words
        p_in = mpl[:cap_p]
        s_lm_in = s_in[s_in < ni]
        if np.intersect1d(p_in, s_lm_in, assume_unique=True).size:
            continue
        s_raw_in = s_in[s_in >= ni]
        if r >= ni and s_raw_in.size and (s_raw_in == r).any():
            continue
        s_whole, p_whole = len(msl) <= cap_s, len(mpl) <= cap_p
        lm_ok = s_whole and p_whole
        if not lm_ok and prefix_rule:
            if s_whole and (len(msl) == 0 or (len(p_in) and msl[-1] <= p_in[-1])):
                lm_ok = True
            if p_whole and (len(mpl) == 0 or (len(s_lm_in) and mpl[-1] <= s_lm_in[-1])):
                lm_ok = True
        if not lm_ok and (len(msl) == 0 or len(mpl) == 0):
            lm_ok = True  # an empty list meets nothing
        raw_ok = r < ni or len(raw) == 0 or len(msl) + len(raw) <= cap_s or (s_raw_in.size and r <= s_raw_in[-1])
        if not (lm_ok and raw_ok):
            dense += 1
    n = max(len(cases), 1)
    lines = (2 if hs > 32 else 1) + (2 if hp > 32 else 1)
    return {"heads": [hs, hp], "mask_bits": mb, "inline": [cap_s, cap_p], "prefix_rule": prefix_rule,
            "dense_pass_share": round(dense / n, 4), "lines_per_request": lines,
            "mean_s_landmarks": round(ls / n, 2), "mean_s_raw": round(lr / n, 2), "mean_p_landmarks": round(lp / n, 2)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", choices=["rbac", "folders", "social"], default="folders")
    p.add_argument("--tuples", type=int, default=5_000_000)
    p.add_argument("--sample", type=int, default=20000)
    p.add_argument("--formats", default="32:32:64,32:32:128,32:32:256,32:16:64,32:16:128,64:32:64,64:32:128,"
                                        "64:32:256,64:32:512,64:64:256,64:64:512,32:32:512",
                   help="HS:HP:mask-bits, comma separated")
    a = p.parse_args()
    w = make(a.workload, a.tuples, a.sample)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    roots, targets = w.resolve(snap)
    li = snap.label_index(32, 32)
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
        lmp = np.union1d(mask_ranks(pm), pl[pl < ni])
        lms = np.union1d(mask_ranks(sm), sl[sl < ni])
        raw = np.sort(sl[sl >= ni])
        cases.append((lmp, lms, raw, r))
    for f in a.formats.split(","):
        hs_, hp_, mb = (int(x) for x in f.split(":"))
        for rule in (True, False) if f == a.formats.split(",")[0] else (True,):
            d = replay(cases, ni, hs_, hp_, mb, rule)
            d.update({"workload": a.workload, "tuples": a.tuples, "requests": len(cases)})
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
