"""Per-launch k_wgrad_h3 durations from a rocprofv3 kernel trace, with what else was resident when each launch
began (the eval chain's kernels on the other queue) -- for the intermittent slow main weight-gradient launches."""
import csv
import glob
import gzip
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv*", recursive=True):
    op = gzip.open if f.endswith(".gz") else open
    rows += list(csv.DictReader(op(f, "rt")))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
for r in rows:
    if "wgrad_h3" not in r["Kernel_Name"]:
        continue
    other = [o for o in rows if o["Queue_Id"] != r["Queue_Id"] and o["s"] < r["e"] and o["e"] > r["s"]]
    desc = ", ".join(o['Kernel_Name'].replace('void ', '').split('(')[0].split('::')[-1][:22]
                     + f"@{(o['s'] - r['s']) / 1e3:+.0f}us" for o in other[:4])
    print(f"h3 {(r['e'] - r['s']) / 1e6:6.3f} ms  beside: {desc}")
