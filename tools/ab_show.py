import glob, json, os, sys
for f in sorted(glob.glob('gpurun_out/ab/b_*.json')):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, 'ERR', e); continue
    st = d.get('stage_ms_per_step', {})
    print(os.path.basename(f), round(d['value']), d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'],
          {k: v for k, v in st.items() if v})
