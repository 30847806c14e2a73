"""Per-kernel mean of PMC counters over the bench-shape dispatches in gpurun_out/pmc_*/."""
import csv, collections, glob, re, sys
rx = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmc_*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        n = re.sub(r"<.*>", "", r['Kernel_Name'].split('(')[0].replace('void ', '').replace('orbfe::', ''))
        if rx and not rx.search(n):
            continue
        key = (n, int(r['Grid_Size']))
        acc[key][r['Counter_Name']].append(float(r['Counter_Value']))
for (n, g), cs in sorted(acc.items()):
    # per dispatch: values are summed over dimensions already; average over dispatches
    out = {c: sum(v) / max(1, len(v)) for c, v in cs.items()}
    # multiple rows per dispatch (per-XCD?) -> count dispatches by SQ_WAVES rows
    print(n, g, {c: round(v) for c, v in sorted(out.items())})
