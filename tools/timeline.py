"""Per-kernel durations of the timed (sub-batch) launches and a window of the two-stream
timeline from gpurun_out/trace_<tag>/ (tools/trace_bench.sh)."""
import collections, csv, glob, sys
tag = sys.argv[1]
sub = int(sys.argv[2]) if len(sys.argv) > 2 else 256
f = glob.glob(f"gpurun_out/trace_{tag}/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbfe::", "").split("<")[0]
    gx, gy = int(r["Grid_Size_X"]), int(r["Grid_Size_Y"])
    if gy == sub or n == "bf_expand_kernel" or (n == "octree_kernel" and gx == sub * int(r["Workgroup_Size_X"])) \
            or (n == "resize_tail_kernel" and gx == sub * int(r["Workgroup_Size_X"])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Queue_Id"]))
ev.sort()
d = collections.defaultdict(list)
for s, e, n, q in ev:
    d[n].append(e - s)
for n, v in sorted(d.items()):
    print(f"{n:28s} {len(v):5d} launches  {sum(v) / len(v) / 1e3:8.1f} us")
w = ev[len(ev) // 2: len(ev) // 2 + int(sys.argv[3]) if len(sys.argv) > 3 else len(ev) // 2 + 30]
t0 = w[0][0]
for s, e, n, q in w:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q} {n}")
