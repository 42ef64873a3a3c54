"""Timeline of host-to-host check calls from a rocprofv3 trace (kernel + memory copy).

    python tools/timeline.py gpurun_out/<dir>/trace [--calls 2] [--match label_kernel]

Reads *kernel_trace.csv and *memory_copy_trace.csv, groups activity into calls (idle gaps
of more than 200 us separate them) and prints, for the last --calls host-to-host calls (a
first stage reading pinned requests in place, `*_host_kernel`, or a pipelined chunk launch),
every kernel and copy relative to the call's first event: the clear, the first stage, the
second / spill stages and the statistics-and-results launch, and the GPU-idle gaps between
them.
"""
import csv
import glob
import os
import sys


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def short(name):
    """the kernel name without namespaces, return type and parameter list"""
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):  # the parameter list starts at the first '(' outside <...>
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return name[:cut][:70]


def main():
    src = sys.argv[1]
    ncalls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 2
    ev = []
    for r in rows(os.path.join(src, "**", "*kernel_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", short(r.get("Kernel_Name", "?"))))
    for r in rows(os.path.join(src, "**", "*memory_copy_trace.csv")):
        kind = r.get("Direction") or r.get("Operation") or r.get("Kind") or "copy"
        size = r.get("Bytes") or r.get("Size") or ""
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", f"{kind} {size}"))
    ev.sort()
    # a run starts with its clear_kernel (results, flags and statistics zeroed); idle gaps of
    # more than 200 us also separate calls
    calls, cur, last_end = [], [], None
    for e in ev:
        if cur and ((last_end is not None and e[0] - last_end > 200_000) or e[3] == "clear_kernel"):
            calls.append(cur)
            cur = []
        cur.append(e)
        last_end = max(last_end or 0, e[1])
    if cur:
        calls.append(cur)
    if "--match" in sys.argv:  # calls with a kernel whose name contains this (e.g. label_kernel: HBM-resident runs)
        m = sys.argv[sys.argv.index("--match") + 1]
        piped = [c for c in calls if any(m in e[3] for e in c)]
    else:
        piped = [c for c in calls if any(", 1>" in e[3] or "_host_kernel" in e[3] for e in c)]
    if "--first" in sys.argv:  # the earliest host-to-host calls (the bench's timed steps)
        piped = piped[:ncalls + 2]
    for c in piped[-ncalls:]:
        t0 = c[0][0]
        end = max(e[1] for e in c)
        print(f"--- call: {len(c)} events, {(end - t0) / 1e3:.1f} us first event to last")
        busy_until = t0
        for s, e, k, name in c:
            gap = (s - busy_until) / 1e3 if k == "K" and s > busy_until else 0.0
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {k} {name}"
                  + (f"   [idle {gap:.1f}]" if gap > 1 else ""))
            if k == "K":
                busy_until = max(busy_until, e)


if __name__ == "__main__":
    main()
