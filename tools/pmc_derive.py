"""Derived per-kernel SQ metrics from tools/pmc_kernels.sh's summary (mean counter value per launch):

    python tools/pmc_derive.py gpurun_out/pmc_r02/summary.txt profiles/r02/pmc_sq.json

  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the share of SIMD-cycles of
                the launch in which the matrix core was busy (SQ_VALU_MFMA_BUSY_CYCLES counts MFMA cycles summed over
                SIMDs; GRBM_GUI_ACTIVE counts GPU-busy cycles summed over the 8 XCDs)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles over all LDS-array cycles)
  wait_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (wave-cycles spent in s_waitcnt)
  valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA
"""
import collections
import json
import sys

c = collections.defaultdict(dict)
for line in open(sys.argv[1]):
    parts = line.split()
    if len(parts) < 3:
        continue
    name, counter, val = " ".join(parts[:-3]) if len(parts) > 4 else parts[0], parts[-3], parts[-2]
    try:
        c[name][counter] = float(val)
    except ValueError:
        continue
out = {}
for k, v in c.items():
    d = {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE"):
        d["mfma_busy"] = round(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    if v.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict"] = round(v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_LDS_IDX_ACTIVE"], 4)
    if v.get("SQ_WAVE_CYCLES"):
        d["wait_frac"] = round(v.get("SQ_WAIT_INST_ANY", 0) / v["SQ_WAVE_CYCLES"], 4)
    if v.get("SQ_INSTS_MFMA"):
        d["valu_per_mfma"] = round(v.get("SQ_INSTS_VALU", 0) / v["SQ_INSTS_MFMA"], 2)
    d["counters"] = v
    out[k] = d
json.dump({"source": sys.argv[1], "definitions": __doc__.split("\n\n")[1].strip(), "kernels": out},
          open(sys.argv[2], "w"), indent=1)
for k, d in sorted(out.items()):
    if "mfma_busy" in d or "gru" in k or "wgrad" in k:
        print(k, {x: y for x, y in d.items() if x != "counters"})
