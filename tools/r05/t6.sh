#!/bin/bash
# Round 5: instruction-cache counters of the GRU kernels (is the 37 KB backward body refetched every step?)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05t6
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -i -E "icache|ifetch|SQC_" $O/avail.txt | head -60 > $O/avail_icache.txt || true
echo "listed"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --kernel-trace -d $O/p1 -o run -- python3 $R/tools/bench_gru.py --which both --iters 1 > $O/p1.log 2>&1
echo "pmc rc=$?"
python3 - $O > $O/summary.txt <<'PY'
import collections, glob, sqlite3, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for db in sorted(glob.glob(f"{out}/*/*.db")):
    c = sqlite3.connect(db)
    try:
        rows = c.execute("select kernel_name, counter_name, value from counters_collection").fetchall()
    except Exception as e:
        print("db error", db, e); continue
    for k, n, v in rows:
        agg[(k.split("(")[0][-40:], n)].append(v)
for (k, n), v in sorted(agg.items()):
    print(f"{k:42s} {n:24s} {sum(v)/len(v):.4g} (n={len(v)})")
PY
cat $O/summary.txt | head -40
cd $R
V=$R/to-ued_amd/exp/libtoued_EVAL_CHOSEN_ROW_1.so
bash tools/gpu_steps.sh r05t6 \
  "tr3:200:TOUED_LIB=$V bash tools/trace_step.sh r05t6_cr" \
  "tr4:200:TOUED_LIB=$V TOUED_EVAL_BLOCK=128 bash tools/trace_step.sh r05t6_crb128"
