"""Per-kernel durations and gaps of the last config-5 calls in gpurun_out/prof_c5 (rocprofv3)."""
import csv, sys
d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_c5'
ev = []
for r in csv.DictReader(open(f'{d}/run_kernel_trace.csv')):
    ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0][:48]))
try:
    for r in csv.DictReader(open(f'{d}/run_memory_copy_trace.csv')):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'COPY ' + r['Direction']))
except FileNotFoundError:
    pass
ev.sort()
idx = [i for i, e in enumerate(ev) if 'fused' in e[2]]
prev = None
for e in ev[idx[-2] - 3:idx[-1] + 12]:
    gap = (e[0] - prev) / 1000 if prev else 0
    print(f"{gap:8.2f} {(e[1] - e[0]) / 1000:8.2f}  {e[2]}")
    prev = e[1]
