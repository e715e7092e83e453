"""Print a bench --clock-json file as a table (ms per sort, avg us, GB/s), largest first."""
import json, sys
d = json.load(open(sys.argv[1]))
tot = sum(v['ms'] for v in d.values())
print(f'total {tot:.1f} ms')
for k, v in sorted(d.items(), key=lambda kv: -kv[1]['ms']):
    if v['ms'] < 0.5: continue
    print(f"{k:45s} {v['ms']:8.2f} ms {100*v['ms']/tot:5.1f}%  n={v['launches']:5d} avg {1e3*v['ms']/v['launches']:8.1f} us  {v['bytes']/v['ms']/1e6:7.0f} GB/s")
