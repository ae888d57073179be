"""Builds librbgpu.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "librbgpu.so")
OBJ = os.path.join(HERE, "build_obj")
ARCH = os.environ.get("RBGPU_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"),
         "-Wall", "-Wno-unused-function"]


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def build(verbose: bool = False, defines=(), out: str = OUT, obj: str = OBJ) -> str:
    """Compiles every csrc/*.hip|*.cpp for gfx950 and links `out`.  `defines` / `out` / `obj` are for
    kernel-variant experiments (scripts/variants.py); the product is the default build."""
    os.makedirs(obj, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.hpp")) + [os.path.join(ROOT, "include", "rbgpu.h")]
    sources = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    objs = []
    jobs = []
    for s in sources:
        o = os.path.join(obj, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer([s] + headers, o):
            dflags = [f"-D{d}" for d in defines]
            cmd = [HIPCC] + FLAGS + dflags + ["-c", s, "-o", o]
            if s.endswith(".cpp"):
                cmd = [HIPCC, "-x", "hip"] + FLAGS + dflags + ["-c", s, "-o", o]
            jobs.append(cmd)

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stderr}")
        return r.stderr

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for err in ex.map(run, jobs):
            if err and verbose:
                print(err, file=sys.stderr)
    if jobs or _newer(objs, out):
        run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs)
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
