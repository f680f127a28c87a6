"""Per-step timeline from a rocprofv3 kernel trace (tools/trace_step.sh): for the last meta-step (between the ends of
the last two k_gru_bwd6n launches), every kernel's queue, start offset and duration, and each queue's busy time."""
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
b = [r for r in rows if "k_gru_bwd6n" in r["Kernel_Name"]]
s0, s1 = b[-2]["e"], b[-1]["e"]
seg = [r for r in rows if s0 <= r["s"] < s1]
print(f"step {(s1 - s0) / 1e6:.3f} ms, {len(seg)} kernels")
busy = collections.defaultdict(float)
for r in seg:
    busy[r["Queue_Id"]] += r["e"] - r["s"]
    if r["e"] - r["s"] > 50000 or r["Queue_Id"] != seg[0]["Queue_Id"]:
        print(f"q{r['Queue_Id']:>2} +{(r['s'] - s0) / 1e6:7.3f} {(r['e'] - r['s']) / 1e6:7.3f} ms  {r['n']}")
for q, v in busy.items():
    print(f"queue {q}: busy {v / 1e6:.3f} ms")
tot = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    tot[r["n"]][0] += 1
    tot[r["n"]][1] += r["e"] - r["s"]
print("per kernel over the step (launches, total ms):")
for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"  {t / 1e6:7.3f} ms  x{c:<3d} {n}")
