"""Build an experimental libtoued_<tag>.so with extra -D flags on one source (timing studies).

    python tools/build_variant.py gru.hip BWD_EXP=1 [...]   -> to-ued_amd/exp/libtoued_BWD_EXP_1.so
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1] / "to-ued_amd"
sys.path.insert(0, str(ROOT))
import build as B  # noqa: E402

srcs = [ROOT / "csrc" / x for x in sys.argv[1].split(",")]   # one source, or several comma-separated
defs = sys.argv[2:]
tag = "_".join(d.replace("=", "_") for d in defs)
out_dir = ROOT / "exp"
out_dir.mkdir(exist_ok=True)
B.build(verbose=False)
cc = B.hipcc()
built = {}
for src in srcs:
    obj = out_dir / f"{src.stem}_{tag}.o"
    subprocess.run([cc, *B._flags(src), *[f"-D{d}" for d in defs], "-c", str(src), "-o", str(obj)], check=True)
    built[src.stem] = obj
objs = [built.get(o.stem, o) for o in (B.OBJ / (s.stem + ".o") for s in sorted(B.CSRC.glob("*.hip")))]
so = out_dir / f"libtoued_{tag}.so"
subprocess.run([cc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(so)], check=True)
print(so)
