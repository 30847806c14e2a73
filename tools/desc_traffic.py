"""Mean describe_kernel HBM traffic per bench-shape launch from two PMC passes:
python tools/desc_traffic.py <fetch_dir> <write_dir> [grid]  (2 x FETCH_SIZE + WRITE_SIZE, KB)."""
import csv
import sys


def per_launch(d, counter, grid=None):
    vals = {}
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        if "describe_kernel" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        if grid and int(r["Grid_Size"]) != grid:
            continue
        vals.setdefault(r["Dispatch_Id"], []).append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    if not vals:
        return None, None
    big = max(g for v in vals.values() for g, _ in v)
    sums = [sum(x for _, x in v) for v in vals.values() if v[0][0] == big]
    return big, sum(sums) / len(sums) * 1024


g, fetch = per_launch(sys.argv[1], "FETCH_SIZE")
_, write = per_launch(sys.argv[2], "WRITE_SIZE", g)
print(f"grid {g}: FETCH {fetch / 1e6:.1f} MB  WRITE {write / 1e6:.1f} MB  traffic {(2 * fetch + write) / 1e6:.1f} MB")
