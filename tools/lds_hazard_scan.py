"""Scan a kernel's gfx950 assembly for the LDS/VMEM store-data hazards behind the lane-half corruption recorded in
DESIGN.md section 7: a VALU instruction that overwrites a VGPR a preceding ds_write / buffer_store still reads as data
within `--window` instructions, and an s_barrier not preceded by `s_waitcnt lgkmcnt(0)` since the last LDS access.

    python tools/lds_hazard_scan.py to-ued_amd/csrc/gru.hip k_gru_bwd6n [--window 4] [--wide]

--wide restricts the store check to stores with a data operand of more than 8 bytes (ds_write_b96/b128,
buffer/global_store_dwordx3/x4; ds_write2_b64 reads two 8-byte operands) -- the stores whose data VGPRs a VALU write may not follow without wait states
(the gfx950 16-byte buffer-store loss in DESIGN.md section 7) -- and flags every VALU write to those VGPRs in the
next --window instructions (hipcc overwrites the data VGPRs of dword and b64 stores 1-3 instructions later as a
matter of course, which the hardware tolerates).
"""
import argparse
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernel")
    ap.add_argument("--window", type=int, default=4)
    ap.add_argument("--wide", action="store_true", help="only stores of more than 8 bytes of data")
    a = ap.parse_args()
    src = Path(a.src)
    out = Path("/tmp") / (src.stem + "_scan.s")
    flags = ["-ffp-contract=fast", "-fno-slp-vectorize"] if src.name in ("gru.hip", "wgrad.hip") else \
        ["-ffp-contract=off"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{ROOT / 'to-ued_amd' / 'csrc'}", *flags, "--cuda-device-only", "-S", str(src), "-o", str(out)],
                   check=True)
    s = out.read_text()
    names = [m.group(1) for m in re.finditer(r"^(_Z\S*" + re.escape(a.kernel) + r"\S*):", s, re.M)]
    bad = 0
    for name in names:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        ins = [l.strip() for l in s[i:j].split("\n") if l.startswith("\t") and not l.strip().startswith((";", "."))]
        pend_lds = False
        for n, t in enumerate(ins):
            op = t.split()[0]
            if op.startswith("ds_"):
                pend_lds = True
            if op == "s_waitcnt" and "lgkmcnt(0)" in t:
                pend_lds = False
            if op == "s_barrier" and pend_lds:
                print(f"{name[:60]}: #{n} s_barrier with LDS accesses not waited for")
                bad += 1
            if op.startswith(("ds_write", "buffer_store", "global_store")):
                wide = op.endswith(("b96", "b128", "dwordx3", "dwordx4"))
                if a.wide and not wide:
                    continue
                ops = [x.strip() for x in t[len(op):].split(",")]
                data = set()
                for x in (ops[1:] if op.startswith("ds_write") else ops[:1]):
                    data |= regs(x.split()[0]) if x else set()
                for q in range(n + 1, min(n + 1 + a.window, len(ins))):
                    u = ins[q]
                    if u.startswith("v_") and not u.startswith(("v_cmp", "v_readfirstlane")):
                        dst = u.split()[1].rstrip(",")
                        if regs(dst) & data:
                            print(f"{name[:60]}: #{n} {t}  ->  +{q - n} {u}")
                            bad += 1
    print(f"{len(names)} kernel(s) scanned, {bad} finding(s) (window {a.window})")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
