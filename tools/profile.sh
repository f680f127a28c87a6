#!/bin/bash
# Profiles committed under profiles/<round>/ come from this script, run on the MI355X box:
#   gpurun -- bash tools/profile.sh r01
# 1) kernel-trace + stats of the headline bench; 2) and 3) separate PMC passes for FETCH_SIZE and
# WRITE_SIZE (one TCC counter group per pass, MI355X_MICROARCH.md "rocprofv3 PMC slots");
# 4) the FETCH/WRITE calibration kernels (tools/calib_fetch.hip) for the counter-to-bytes factors.
set -euo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 "$R/tools/calib_fetch.hip" -o /tmp/calib_fetch 2>/dev/null
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d "$OUT/ks" -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 \
    --no_cpu_baseline --workloads none > "$OUT/ks.log" 2>&1
echo "kernel-trace done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d "$OUT/ks_wl" -o run -- python3 "$R/bench.py" --steps 2 \
    --warmup 1 --no_cpu_baseline --workloads c3,c4 > "$OUT/ks_wl.log" 2>&1
echo "workloads kernel-trace done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" \
    --steps 1 --warmup 1 --no_cpu_baseline --workloads none > "$OUT/pmc_fetch.log" 2>&1
echo "fetch pass done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" \
    --steps 1 --warmup 1 --no_cpu_baseline --workloads none > "$OUT/pmc_write.log" 2>&1
echo "write pass done"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/calib_fetch" -o run -- /tmp/calib_fetch \
    > "$OUT/calib_fetch.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/calib_write" -o run -- /tmp/calib_fetch \
    > "$OUT/calib_write.log" 2>&1
echo "calibration done"
# summarise on the box (kernel_stats*.csv, pmc_traffic.json) and drop the databases: gpurun copies back <= 64 MiB
python3 "$R/tools/prof_summary.py" "$OUT" "$R/gpurun_out/prof_${TAG}_summary" && find "$OUT" -name "*.db" -delete
find "$OUT" -name "*kernel_trace.csv" -delete
ls -la "$R/gpurun_out/prof_${TAG}_summary"
