"""Build libsemops.so (HIP kernels for gfx950 + C ABI) in-tree.

The shared library lands in sem_amd/lib/ so it travels with the repository
snapshot to the GPU box; no JIT cache, no site-packages install.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
# SEM_LIBDIR: another in-tree output directory (e.g. sem_amd/lib_diag for a diagnostic build beside the
# release one, tools/kbench.py ablations); default sem_amd/lib
LIBDIR = os.environ.get("SEM_LIBDIR") or os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libsemops.so")
ARCH = os.environ.get("SEM_OFFLOAD_ARCH", "gfx950")

SOURCES = ["sem_ops.hip", "apply_band.hip", "gll_tables.cpp", "krylov_sweeps.hip", "ns_velocity.hip", "ns_apply.hip", "block_gemv.hip", "ns_condense.hip",
           "dense_inverse.hip", "front_solve.hip"]
HEADERS = ["sem_internal.h", "gll_consts.h", "apply_common.h", os.path.join("..", "..", "include", "sem_ops.h")]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the SEM operator layer needs ROCm's hipcc to build")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


def source_hash():
    """Hash of every source and header of the library (and this build script), embedded in the
    library as sem_build_id(); sem_amd._lib refuses a library built from other sources."""
    import hashlib
    h = hashlib.sha256()
    for name in sorted(SOURCES + HEADERS) + [os.path.join("..", "build.py")]:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read() + b"\0")
    return h.hexdigest()[:16]


CONSTS = os.path.join(CSRC, "gll_consts.h")


def gen_consts(verbose=False):
    """Regenerate gll_consts.h (compile-time GLL tables) with the host GLL code."""
    exe = os.path.join(LIBDIR, "gen_consts")
    cxx = shutil.which("g++") or _hipcc()
    cmd = [cxx, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"), "-o", exe,
           os.path.join(CSRC, "gen_consts.cpp"), os.path.join(CSRC, "gll_tables.cpp")]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    text = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    old = open(CONSTS).read() if os.path.exists(CONSTS) else None
    if text != old:
        with open(CONSTS, "w") as f:
            f.write(text)
    return CONSTS


# Per-source flags.  apply_band.hip: the command processor preloads the first 14 kernel-argument
# SGPRs (the scalar prologue arguments of apply_band_kp), so a tile's first global load does not
# wait on a kernarg memory fetch.  The code object keeps a fallback prologue that loads them itself
# when the firmware does not preload.
EXTRA_FLAGS = {"apply_band.hip": ["-mllvm", "-amdgpu-kernarg-preload-count=14"]}


def build(force=False, verbose=False, diag=False):
    """diag=True: a diagnostic build (SEM_DIAGNOSTICS=1: SEM_DIAG ablation bits and per-wave phase
    stamps, for tools/kbench.py); its build id carries "+diag" and sem_amd._lib loads it only with
    SEM_ALLOW_DIAG=1.  The default build has no diagnostic path at all."""
    mode = "diag" if diag else "release"
    stamp = os.path.join(LIBDIR, ".build_mode")
    prev_mode = open(stamp).read().strip() if os.path.exists(stamp) else None
    force = force or prev_mode != mode
    if not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    gen_consts(verbose)
    hipcc = _hipcc()
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-I", os.path.join(ROOT, "include"),
             f"-DSEM_DIAGNOSTICS={1 if diag else 0}"]
    objs, procs = [], []
    hdr_t = max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS + [os.path.join("..", "build.py")])
    bid = source_hash()
    for src in SOURCES:  # one hipcc per translation unit, in parallel; unchanged objects are reused
        obj = os.path.join(LIBDIR, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        # the build id goes into the small host TU only, so a source change rebuilds just that TU
        # and the changed one; it is recompiled on every build
        extra = [f'-DSEM_BUILD_ID="{bid}"'] if src == "gll_tables.cpp" else []
        if (not force and not extra and os.path.exists(obj)
                and os.path.getmtime(obj) > max(hdr_t, os.path.getmtime(os.path.join(CSRC, src)))):
            continue
        cmd = [hipcc] + flags + extra + EXTRA_FLAGS.get(src, []) + ["-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((src, subprocess.Popen(cmd)))
    bad = [src for src, pr in procs if pr.wait() != 0]
    if bad:
        raise RuntimeError(f"hipcc failed on {bad}")
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    with open(stamp, "w") as f:
        f.write(mode)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv)
    print(LIB)
