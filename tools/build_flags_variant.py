"""Build an experimental libtoued_<tag>.so from one source with its compile flags edited (timing studies):

    python tools/build_flags_variant.py gru.hip <tag> [-flag-to-drop ...] [+flag-to-add ...]
    -> to-ued_amd/exp/libtoued_<tag>.so
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1] / "to-ued_amd"
sys.path.insert(0, str(ROOT))
import build as B  # noqa: E402

src = ROOT / "csrc" / sys.argv[1]
tag = sys.argv[2]
drop = [a[1:] for a in sys.argv[3:] if a.startswith("-")]
add = [a[1:] for a in sys.argv[3:] if a.startswith("+")]
out_dir = ROOT / "exp"
out_dir.mkdir(exist_ok=True)
B.build(verbose=False)
cc = B.hipcc()
obj = out_dir / f"{src.stem}_{tag}.o"
flags = [f for f in B._flags(src) if f not in drop] + add
subprocess.run([cc, *flags, "-c", str(src), "-o", str(obj)], check=True)
objs = [obj if o.stem == src.stem else o for o in (B.OBJ / (s.stem + ".o") for s in sorted(B.CSRC.glob("*.hip")))]
so = out_dir / f"libtoued_{tag}.so"
subprocess.run([cc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(so)], check=True)
obj.unlink()
print(so)
