"""Timeline of the last C3 regret round in a rocprofv3 kernel trace of tools/regret_round.py: the rounds are the
trace's kernel runs separated by host gaps > 1 ms (each round ends in a synchronize and a print).

    rocprofv3 --kernel-trace --output-format csv -d <dir> -o run -- python3 tools/regret_round.py 3
    python3 tools/round_timeline.py <dir>
"""
import collections
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
rows.sort(key=lambda r: r["s"])
# rounds: from one k_key_chain launch (the antagonists' update keys, early in each round) to the next
kc = [i for i, r in enumerate(rows) if "k_key_chain" in r["Kernel_Name"]]
segs = [rows[a:b] for a, b in zip(kc, kc[1:])] or [rows]
seg = segs[-1]
s0 = seg[0]["s"]
print(f"{len(segs)} rounds between k_key_chain launches; last: {(max(r['e'] for r in seg) - s0) / 1e6:.3f} ms, {len(seg)} kernels")
busy = collections.defaultdict(float)
for r in seg:
    busy[r["Queue_Id"]] += r["e"] - r["s"]
    if r["e"] - r["s"] > 30000:
        print(f"q{r['Queue_Id']:>2} +{(r['s'] - s0) / 1e6:7.3f} {(r['e'] - r['s']) / 1e6:7.3f} ms  {r['n']}")
for q, v in busy.items():
    print(f"queue {q}: busy {v / 1e6:.3f} ms")
tot = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    tot[r["n"]][0] += 1
    tot[r["n"]][1] += r["e"] - r["s"]
print("per kernel over the round (launches, total ms):")
for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"  {t / 1e6:7.3f} ms  x{c:<3d} {n}")
