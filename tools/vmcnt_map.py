"""Find the memory waits a kernel's register pressure costs it: every scratch reload followed closely by an
`s_waitcnt vmcnt(0)` (the reload drains every outstanding buffer load AND store, vmcnt counts both on gfx9),
and every waterfall loop (v_readfirstlane + v_cmp_eq: a lane-dependent buffer soffset or descriptor).

    python tools/vmcnt_map.py gru.hip k_gru_bwd6n [-DNAME=V ...]
"""
import re
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
src, kern, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
subprocess.run([sys.executable, str(HERE / "spill_map.py"), src, kern, *defs], stdout=subprocess.DEVNULL, check=True)
s = Path("/tmp/spill_map.s").read_text()
m = re.search(r"^(\S*" + kern + r"\S*):", s, re.M)
body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
loc, ins = None, []
for line in body:
    mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
    if mm:
        loc = int(mm.group(2))
        continue
    if line.strip() and not line.strip().startswith((".", ";")):
        ins.append((loc, line.strip()))
print(f"{kern}: scratch ops {sum('scratch_' in l for _, l in ins)}, vmcnt(0) waits {sum('vmcnt(0)' in l for _, l in ins)}")
for i, (lc, l) in enumerate(ins):
    if "scratch_load" in l:
        for j in range(i + 1, min(i + 25, len(ins))):
            if "vmcnt(0)" in ins[j][1]:
                print(f"  reload at line {lc} -> vmcnt(0) {j - i} instructions later, before line {ins[j + 1][0]}: "
                      f"{ins[j + 1][1][:60]}")
                break
    if "v_readfirstlane" in l and i + 1 < len(ins) and "v_cmp_eq" in ins[i + 1][1]:
        print(f"  waterfall at line {lc}: {l}")
ps = re.search(re.escape(m.group(1)) + r"\.private_seg_size, (\d+)", s)
print(f"  private segment {ps.group(1) if ps else '?'} bytes")
