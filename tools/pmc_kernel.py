"""Mean PMC counter value per launch of the kernels matching a prefix, from rocprofv3 databases (A/B runs).

    python tools/pmc_kernel.py FETCH_SIZE k_wgrad_h3 gpurun_out/x/pmc0 gpurun_out/x/pmc2
"""
import glob
import sqlite3
import sys
from collections import defaultdict

counter, prefix, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
for d in dirs:
    agg = defaultdict(list)
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        for name, val in c.execute("select kernel_name, value from counters_collection where counter_name = ?",
                                   (counter,)):
            n = name.replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0]
            if n.startswith(prefix):
                agg[n].append(float(val))
    for n, v in agg.items():
        print(f"{d}: {n}: {counter} mean {sum(v) / len(v):.6g} over {len(v)} launches")
