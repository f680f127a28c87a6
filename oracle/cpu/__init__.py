"""C++/OpenMP CPU restatement of the rollout + GAE + A2C update (test infrastructure and the bench's CPU baselines).

build() compiles rollout_cpu.cpp with g++ -O3 -fopenmp -ffp-contract=off into librollout_cpu.so next to it;
lib() loads it (building on demand).  Only tests/, bench.py's cpu_baseline and __graft_entry__ use it.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "rollout_cpu.cpp"
SO = HERE / "librollout_cpu.so"
_lib = None


def build(force: bool = False) -> Path:
    if force or not SO.exists() or SO.stat().st_mtime < SRC.stat().st_mtime:
        cmd = ["g++", "-O3", "-march=x86-64-v2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-std=c++17",
               "-shared", "-fPIC", str(SRC), "-o", str(SO)]
        subprocess.run(cmd, check=True)
    return SO


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(SO))
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.toued_cpu_rollout.argtypes = [I, I, I, I, P, P, I, P, P, I, I, I, P, P, P, P, P, P]
        L.toued_cpu_gae.argtypes = [P, I, P, P, P, P, I, I, I, F, F, P, P]
        L.toued_cpu_a2c_update.argtypes = [P, P, P, P, I, P, P, P, P, P, I, I, I, F, F, F, F, F, F, P]
        L.toued_cpu_threads.argtypes = []
        _lib = L
    return _lib


def threads() -> int:
    """the OpenMP team size the library runs with (OMP_NUM_THREADS or the host's cores)"""
    return int(lib().toued_cpu_threads())
