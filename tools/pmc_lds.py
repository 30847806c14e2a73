#!/usr/bin/env python3
"""LDS pressure per kernel from one PMC pass (tools/pmc_kernel.sh with SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS
SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE):
python tools/pmc_lds.py gpurun_out/pmc_SQ_LDS_BANK_CONFLICT_lds [out.json]"""
import collections
import csv
import json
import re
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
    n = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbfe::", ""))
    acc[(n, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for (n, g), cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    idx, bc = m.get("SQ_LDS_IDX_ACTIVE", 0), m.get("SQ_LDS_BANK_CONFLICT", 0)
    # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (one GPU-active count per XCD): per XCD
    gui = m.get("GRBM_GUI_ACTIVE", 8) / 8
    out[f"{n}[{g}]"] = {
        "conflict_cycles_per_access_cycle": round(bc / max(1.0, idx - bc), 4),
        # per-CU shares of the kernel's GPU-active cycles (256 CUs)
        "lds_idx_active_pct": round(100 * idx / gui / 256, 1),
        "lds_bank_conflict_pct": round(100 * bc / gui / 256, 1),
        "addr_conflict": m.get("SQ_LDS_ADDR_CONFLICT", 0),
        "unaligned_stall": m.get("SQ_LDS_UNALIGNED_STALL", 0),
        "active_inst_lds": m.get("SQ_ACTIVE_INST_LDS", 0),
        "active_inst_valu": m.get("SQ_ACTIVE_INST_VALU", 0),
        "wait_inst_lds": m.get("SQ_WAIT_INST_LDS", 0),
        "busy_cu_cycles": m.get("SQ_BUSY_CU_CYCLES", 0),
        "gui_active": gui,
        "dispatches": len(cs.get("GRBM_GUI_ACTIVE", [])),
    }
    o = out[f"{n}[{g}]"]
    print(f"{n[:24]:24s} {g:>10d} conflicts/access {o['conflict_cycles_per_access_cycle']:.3f} "
          f"LDS idx active {o['lds_idx_active_pct']:5.1f}% bank-conflict {o['lds_bank_conflict_pct']:5.1f}%")
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
