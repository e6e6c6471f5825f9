import json, sys, glob, os
d0 = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d0, '*.log'))):
    try:
        l = [x for x in open(f) if x.startswith('{')][-1]
    except IndexError:
        print(os.path.basename(f), 'no result'); continue
    d = json.loads(l)
    print(f"{os.path.basename(f):14s} {d['value']:>12.0f} {d['ms_per_step']:7.3f} fin={d['stage_ms']['final']:.3f} msm={d['stage_ms']['msm']:.3f} lat={d['batch_latency_ms']:.3f} frac={d['roofline']['frac']:.4f}")
