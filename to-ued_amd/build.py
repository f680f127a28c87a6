"""Build libtoued_hip.so for gfx950 (in-tree, so it travels with the repo snapshot).

    python to-ued_amd/build.py [--force] [--jobs N]

Every .hip file under csrc/ is compiled to an object with hipcc
(--offload-arch=gfx950), then linked into toued/libtoued_hip.so.  Files whose
results must be bit-identical to the CPU oracle (env, PRNG, level generator,
agent maths) are compiled with -ffp-contract=off; the MFMA GRU kernels allow
contraction.  Objects are rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
OUT = ROOT / "toued" / "libtoued_hip.so"
ARCH = os.environ.get("TOUED_ARCH", "gfx950")

# files allowed to contract a*b+c into fma (tolerance-checked float kernels)
CONTRACT_OK = {"gru.hip"}
# per-file extras: packed f32 VALU (SLP-vectorised adds) beside MFMAs costs issue cycles (MI355X_MICROARCH.md)
EXTRA = {"wgrad.hip": ["-fno-slp-vectorize"], "gru.hip": ["-fno-slp-vectorize"]}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (set HIPCC)")


def _flags(src: Path):
    f = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", "-munsafe-fp-atomics"]
    f.append("-ffp-contract=fast" if src.name in CONTRACT_OK else "-ffp-contract=off")
    f += EXTRA.get(src.name, [])
    return f


def _stale(obj: Path, src: Path, headers) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in headers)


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> Path:
    srcs = sorted(CSRC.glob("*.hip"))
    headers = sorted(CSRC.glob("*.h"))
    OBJ.mkdir(parents=True, exist_ok=True)
    cc = hipcc()
    todo = [s for s in srcs if force or _stale(OBJ / (s.stem + ".o"), s, headers)]

    def compile_one(src: Path):
        obj = OBJ / (src.stem + ".o")
        cmd = [cc, *_flags(src), "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return src.name

    if todo:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            for name in ex.map(compile_one, todo):
                if verbose:
                    print(f"[toued build] compiled {name}", flush=True)
    objs = [OBJ / (s.stem + ".o") for s in srcs]
    if todo or not OUT.exists() or any(o.stat().st_mtime > OUT.stat().st_mtime for o in objs):
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(OUT)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[toued build] linked {OUT}", flush=True)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    build(a.force, a.jobs)
    sys.exit(0)
