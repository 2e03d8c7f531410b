"""Summarise tools/gpu_ab_g.sh output: per build, the mapped hand-off ms per config and the C5
ids bench G idx/s (when run)."""
import glob, json, os, sys
d = sys.argv[1]
names = sorted({os.path.basename(f).rsplit('_', 1)[0] for f in glob.glob(d + '/*_h*.json')})
for n in names:
    hs = [json.loads(open(f).read().strip().split('\n')[-1]) for f in sorted(glob.glob(f'{d}/{n}_h*.json'))]
    line = f"{n:8s}"
    for c in hs[0]:
        line += f" {c} ms " + ' '.join('%.4f' % h[c]['ms_per_epoch'] for h in hs)
    b = [json.load(open(f)) for f in sorted(glob.glob(f'{d}/{n}_b*.json'))]
    if b:
        line += (f"   ids G idx/s {' '.join('%.1f' % x['value'] for x in b)}"
                 f"   kernel TB/s {' '.join('%.2f' % (x['roofline']['achieved'] / 1000) for x in b)}")
    print(line)
