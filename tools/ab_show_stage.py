"""Print value, ms/step and per-stage times of bench lines: python tools/ab_show_stage.py FILES..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    st = d.get("stage_ms_per_step", {})
    print(f"{f:40s} {d['value']:10.0f} {d['ms_per_step']:7.3f} ms  " +
          " ".join(f"{k}={v:.4f}" for k, v in st.items() if v))
