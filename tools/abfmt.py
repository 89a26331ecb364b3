import json, sys
for l in sys.stdin:
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{d['workload']:16s} {d['variant']:24s} {d['ms']*1e3:8.1f} us  spread {d['spread']}")
    elif l:
        print(l[:200])
