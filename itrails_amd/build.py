"""Build libitrails_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension:
the library is a plain C-ABI shared object so it travels with the repository snapshot)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["hmm_sweeps.hip", "mfma_sweeps.hip", "wave_sweeps.hip", "dense.hip", "vanloan.hip", "emission.hip", "rows.hip", "prune_vit.hip", "maf.cpp", "writers.cpp", "planner.cpp", "host_io.cpp", "capi.cpp"]
OUT = os.path.join(HERE, "libitrails_hip.so")
# The sweeps never produce NaN (log 0 = -inf is the only non-finite value, and no
# inf - inf or 0/0 is formed), so fmax needs no NaN-quieting canonicalize after each DPP
# move; infinities keep their IEEE semantics (no -ffinite-math-only).
EXTRA = {"hmm_sweeps.hip": ["-fno-honor-nans"], "mfma_sweeps.hip": ["-fno-honor-nans"], "wave_sweeps.hip": ["-fno-honor-nans"],
         "prune_vit.hip": ["-fno-honor-nans"]}
ARCH = os.environ.get("ITR_OFFLOAD_ARCH", "gfx950")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "itrails_hip.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, diag: bool = False,
          variant: str = "", extra_flags=None) -> str:
    """variant: an experiment build (libitrails_hip_<variant>.so, extra flags from
    ITR_HIPCC_FLAGS), loaded with ITR_LIB; never the product library."""
    out = OUT if not diag else OUT.replace(".so", "_diag.so")
    if variant:
        out = OUT.replace(".so", f"_{variant}.so")
    if not force and not diag and not variant and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-fvisibility=hidden"] + (extra_flags if extra_flags is not None else
                                       os.environ.get("ITR_HIPCC_FLAGS", "").split())
    if diag:
        flags += ["-DITR_DIAG"]
    tag = "_diag" if diag else (f"_{variant}" if variant else "")
    objs, procs = [], []
    for src in SOURCES:  # one compiler per translation unit, in parallel
        obj = os.path.join(CSRC, "..", f".{os.path.splitext(src)[0]}{tag}.o")
        cmd = [hipcc] + flags + EXTRA.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    rcs = [p.wait() for p in procs]
    if any(rcs):
        raise subprocess.CalledProcessError(max(rcs), "hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    for o in objs:
        os.remove(o)
    return out


def build_blocks_ext(force: bool = False, verbose: bool = False) -> str:
    """itrails_amd/_blocks*.so: the CPython extension that scans a V_lst's int64 arrays for
    the host-block entry points (csrc/blocks_ext.c; gcc against this interpreter's headers)."""
    import sysconfig

    import numpy as np
    src = os.path.join(CSRC, "blocks_ext.c")
    out = os.path.join(HERE, "_blocks" + sysconfig.get_config_var("EXT_SUFFIX"))
    if not force and os.path.exists(out) and os.path.getmtime(out) > os.path.getmtime(src):
        return out
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-shared", "-fPIC", "-Wall",
           "-I" + sysconfig.get_paths()["include"], "-I" + np.get_include(), src,
           "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    if "--with-exp" in sys.argv:  # product + experiment library (env knobs), in parallel
        import threading
        t = threading.Thread(target=lambda: print(build(force=True, extra_flags=[])))
        t.start()
        print(build(variant="exp", extra_flags=["-DITR_EXPERIMENT"]))
        t.join()
    else:
        print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
        if "--diag" not in sys.argv:
            print(build_blocks_ext(force="--force" in sys.argv, verbose=True))
