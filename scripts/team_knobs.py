import json, os, sys
sys.path.insert(0, '.')
from scripts.lstm_latency import bench
for k in (0, 256, 512, 768, 8, 16, 32, 512 + 8):
    os.environ['DCA_TEAM_KNOBS'] = str(k)
    r = bench(8, 700, 512, reps=3, impl='team')
    print(json.dumps({'knobs': k, 'fwd': r['fwd_us_per_step'], 'err': r['err']}), flush=True)
