import csv, glob, sys, os
src = sys.argv[1]
ev = []
for p in glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        n = n[:n.find("(")] if "(" in n else n
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", n[:60]))
for p in glob.glob(os.path.join(src, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", (r.get("Direction") or "") + " " + (r.get("Bytes") or r.get("Size") or "")))
ev.sort()
calls, cur = [], []
for e in ev:
    if cur and e[0] - max(x[1] for x in cur) > 150000:
        calls.append(cur); cur = []
    cur.append(e)
calls.append(cur)
want = sys.argv[2] if len(sys.argv) > 2 else "host_kernel"
hc = [c for c in calls if any(want in x[3] for x in c)]
print(len(calls), "calls,", len(hc), "with", want)
for c in hc[-3:-1]:
    t0 = c[0][0]
    print("--- call span %.1f us" % ((max(x[1] for x in c) - t0) / 1e3))
    for s, e, k, n in c:
        print("  %8.1f %8.1f  %7.1f us  %s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, k, n))
