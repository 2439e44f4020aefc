"""Per-kernel summary of an ab.sh run: python tools/abshow.py gpurun_out/ab_TAG
(value, k_xspec / k_moments avg launch ms, k_tr_mom / k_postfit totals, stage ms)."""
import json,sys,glob
for f in sorted(glob.glob(sys.argv[1]+'/*.json')):
    try: d=json.loads([l for l in open(f) if l.startswith('{')][-1])
    except Exception as e: print(f, 'ERR'); continue
    k=d.get('kernels',{}); sf=(d.get('solver_fp64') or {}).get('kernels',{})
    print('%-45s %10.1f xs %.3f mom %s tr %s pf %s st %s' % (f.split('/')[-1][:45], d['value'], k.get('xspec',{}).get('avg_launch_ms',0), round(k.get('moments',{}).get('avg_launch_ms',0),3), sf.get('tr_mom',{}).get('total_ms'), sf.get('postfit',{}).get('total_ms'), {a:round(b,1) for a,b in (d.get('stage_ms') or {}).items()}))
