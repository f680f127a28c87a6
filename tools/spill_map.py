"""Map a kernel's scratch spill/reload instructions to source lines (register-pressure work).

    python tools/spill_map.py gru.hip k_gru_bwd6n [-DNAME=V ...]
"""
import collections
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1] / "to-ued_amd"
src, kern, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
out = Path("/tmp/spill_map.s")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-gline-tables-only",
                f"-I{ROOT / 'csrc'}", "--cuda-device-only", "-S", *defs, str(ROOT / "csrc" / src), "-o", str(out)],
               check=True)
s = out.read_text()
m = re.search(r"^(\S*" + kern + r"\S*):", s, re.M)
body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
files = {int(a): b for a, b in re.findall(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', s)}
loc, cnt = None, collections.Counter()
for line in body:
    mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
    if mm:
        loc = (files.get(int(mm.group(1)), mm.group(1)), int(mm.group(2)))
        continue
    if "scratch_store" in line or "scratch_load" in line:
        cnt[("store" if "store" in line else "load", loc)] += 1
for (k, lc), n in sorted(cnt.items(), key=lambda x: (x[0][1] or ("", 0))[1]):
    print(f"{k:5s} {lc[0] if lc else '?'}:{lc[1] if lc else '?'} x{n}")
print("total", sum(cnt.values()))
