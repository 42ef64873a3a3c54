"""Summarise the rocprofv3 output of tools/profile.sh into profiles/<tag>/.

    python tools/pmc_traffic.py gpurun_out/prof_<tag> profiles/<tag> [--workload config2_rbac]

Reads the kernel-trace stats (trace/**/*kernel_stats.csv, *kernel_trace.csv) and one
--pmc directory per counter pass (pmc_*/**/*counter_collection.csv) and writes
  kernel_stats.csv   the rocprofv3 --stats summary, copied as is
  traffic.json       per kernel family: average duration (kernel trace), resources of the
                     dispatch, per-dispatch average of every counter, and HBM bytes per
                     launch from FETCH_SIZE/WRITE_SIZE (KB in rocprofv3) — raw, and with
                     FETCH_SIZE doubled as MI355X_MICROARCH.md "HBM" prescribes for gfx950
                     (128-B read requests tallied at 64 B).  bench.py reads
                     kernels[<family>].hbm_bytes_per_launch for roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

FAMILIES = [
    # host batches with pinned requests: the first stage reading its requests in place
    ("bidi_host_kernel (host batches)", r"bidi_host_kernel"),
    # plan label: closure labels (one intersection per request)
    ("label_host_kernel (host batches)", r"label_host_kernel"),
    ("label_rest_kernel (second stage)", r"label_rest_kernel"),
    ("label_full_kernel (overflow lists)", r"label_full_kernel"),
    ("label_kernel", r"\blabel_kernel"),
    # plan core: lite over the core arrays with closure rows (template argument CL = true)
    ("core lite_host_kernel (host batches)", r"lite_host_kernel<.*, true>"),
    ("core lite_kernel", r"\blite_kernel<.*, true>"),
    ("lite_host_kernel (host batches)", r"lite_host_kernel"),
    ("lite_kernel", r"\blite_kernel"),
    # the pipelined host-to-host first stage is its own instantiation (last template
    # argument 1), so a launch per chunk never mixes into the full-batch launch's figures
    ("bidi_kernel<16> (pipelined chunks)", r"bidi_kernel<16, 9, .*, 1>"),
    ("bidi_kernel<16>", r"bidi_kernel<16, 9, "),
    ("bidi spill stage w (16 requests, 2048 slots)", r"bidi_kernel<16, 11, "),
    ("bidi spill stage h (16 requests, 1024 slots)", r"bidi_kernel<16, 10, "),
    ("bidi spill stage q/r (4 requests)", r"bidi_kernel<4, "),
    ("bidi single-request stage", r"bidi_kernel<1, 13, "),
    ("unit2_kernel<16>", r"unit2_kernel<16>"),
    ("unit2_kernel<4>+<1> (spill passes)", r"unit2_kernel<(4|1)>"),
    ("unit_kernel", r"[^2]unit_kernel<"),
    ("expand_kernel", r"\bexpand_kernel"),
    ("pull_kernel", r"\bpull_kernel"),
    ("reset_kernel", r"\breset_kernel"),
    ("gather_kernel", r"\bgather_kernel"),
    ("seed_kernel", r"\bseed_kernel"),
    ("part_expand_kernel", r"part_expand_kernel"),
    ("part_apply_kernel", r"part_apply_kernel"),
    ("part_gather_kernel", r"part_gather_kernel"),
    ("part_reset_kernel", r"part_reset_kernel"),
    ("part_pull_answer_kernel", r"part_pull_answer_kernel"),
    # two-tier partitioned engine (config #5)
    ("tier_label_kernel", r"tier_label_kernel"),
    ("tier_label exchange kernels (pairs, replies, lengths, bounds)",
     r"tier_pair_kernel|tier_label_reply|tier_label_lens|tier_label_bounds"),
    ("tier_eval_kernel", r"tier_eval_kernel"),
    ("tier_cascade_kernel", r"tier_cascade_kernel"),
    ("tier_seed_kernel", r"tier_seed_kernel"),
    ("tier_query kernels (count + scatter)", r"tier_query_"),
    ("tier_reply kernels (len + scan + copy)", r"tier_reply_|tier_scan_"),
]


def family(name):
    for fam, rx in FAMILIES:
        if re.search(rx, name):
            return fam
    return None


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def summarise(src, workload):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from keto_amd.build import kernel_source_hash
    # the kernel sources this profile was taken at: bench.py reports the traffic only
    # while they are unchanged
    out = {"workload": workload, "source": src, "source_hash": kernel_source_hash(), "kernels": {}}
    # Per family, only the dispatches of its most frequent grid size are averaged: a run
    # also launches the same kernel over smaller batches (trials, chunks, tails), whose
    # per-launch bytes and durations would otherwise be mixed into the bench's launch.
    def grid(r):  # total work-items (kernel trace: Grid_Size_X/Y/Z; counter collection: Grid_Size)
        if "Grid_Size_X" in r:
            return str(int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1))
        return r.get("Grid_Size", "")

    grids = defaultdict(lambda: defaultdict(int))
    rows = []
    for tr in glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in read_csv(tr):
            fam = family(r.get("Kernel_Name", ""))
            if fam:
                rows.append((fam, r))
                grids[fam][grid(r)] += 1
    modal = {fam: max(g, key=g.get) for fam, g in grids.items()}
    dur = defaultdict(list)
    res = {}
    for fam, r in rows:
        if grid(r) != modal[fam]:
            continue
        dur[fam].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        res[fam] = {k: r[k] for k in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size",
                                      "Workgroup_Size") if k in r}
        res[fam]["grid_size"] = modal[fam]
    per = defaultdict(lambda: defaultdict(list))
    for cc in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        by_dispatch = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in read_csv(cc):
            fam = family(r.get("Kernel_Name", ""))
            if not fam:
                continue
            if fam in modal and grid(r) != modal[fam]:
                continue
            d = (cc, r.get("Dispatch_Id"), r.get("Agent_Id"))
            by_dispatch[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = fam
        for d, ctrs in by_dispatch.items():
            for c, v in ctrs.items():
                per[names[d]][c].append(v)
    for fam in sorted(set(per) | set(dur)):
        k = {"dispatches_timed": len(dur.get(fam, []))}
        if dur.get(fam):
            k["avg_duration_ms"] = sum(dur[fam]) / len(dur[fam]) / 1e6
        k["resources"] = res.get(fam)
        c = {n: sum(v) / len(v) for n, v in sorted(per[fam].items())}
        k["counters"] = c
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            k["hbm_bytes_per_launch_raw"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            k["hbm_bytes_per_launch"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            if k.get("avg_duration_ms"):
                k["hbm_GBps"] = k["hbm_bytes_per_launch"] / (k["avg_duration_ms"] * 1e-3) / 1e9
        if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
            k["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if c.get("SQ_WAVE_CYCLES", 0) > 0:
            for part in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if part in c:
                    k[part.lower() + "_frac"] = c[part] / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_WAVES", 0) > 0:  # instructions per wave (one wave = one unit for the bidi kernels)
            for part in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM"):
                if part in c:
                    k[part.lower() + "_per_wave"] = c[part] / c["SQ_WAVES"]
        if c.get("SQ_INSTS_VALU") and k.get("avg_duration_ms"):
            # VALU issue share: a wave64 VALU instruction holds its SIMD's VALU for 4 cycles;
            # 1024 SIMDs at 2.4 GHz (MI355X_MICROARCH.md)
            k["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 4 / (1024 * 2.4e9 * k["avg_duration_ms"] * 1e-3)
        out["kernels"][fam] = k
    out["note"] = ("FETCH_SIZE/WRITE_SIZE are KB per dispatch; hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                   "(gfx950 read correction, MI355X_MICROARCH.md 'HBM'); *_raw without the doubling.  The counters "
                   "sit at the L2's memory side, so Infinity-Cache hits are included.")
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    workload = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "config2_rbac"
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    out = summarise(src, workload)
    with open(os.path.join(dst, "traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({fam: {kk: v.get(kk) for kk in ("avg_duration_ms", "hbm_bytes_per_launch", "hbm_GBps",
                                                      "l2_hit_rate")}
                      for fam, v in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
