"""Average kernel durations from a rocprofv3 rocpd database: python tools/ktime.py DB [substring ...]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pats = sys.argv[2:]
agg = collections.defaultdict(list)
for name, dur in c.execute("select name, duration from kernels"):
    n = name.replace("(anonymous namespace)::", "")
    n = (n[5:] if n.startswith("void ") else n).split("(")[0][:60]
    if not pats or any(p in n for p in pats):
        agg[n].append(dur)
for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f"{k:62s} {len(v):4d} {sum(v) / len(v) / 1e3:10.1f} us")
