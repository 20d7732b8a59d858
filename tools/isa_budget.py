"""Static instruction budget of a band-kernel instantiation by phase.

Compiles sem_amd/csrc/apply_band.hip for gfx950 to assembly (device only, P = 8 instantiations, a scratch copy in
/tmp), cuts the chosen kernel at its two s_barrier instructions -- prologue (tile map, staging, pointwise loads),
roles (the X and Y contractions: all four role paths, of which a wave runs one), epilogue (combination, Dirichlet
rows, stores) -- and counts VALU (fp64 FMA/add/mul separately), SALU, LDS, VMEM and waitcnt per section; the role
section is also split per role path at its branch targets when --paths is given.  Alongside: the even-odd plan's
fp64 operation count per wave (the arithmetic the contraction needs), so the overhead is explicit.

    python tools/isa_budget.py [--kernel 'apply_band_kp<8, 1, 8, 2, false, 0, true>'] [--asm FILE]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mangle(P, TXE, TYE, NS, full, cm, grad):
    b = lambda v: "Lb1E" if v else "Lb0E"  # noqa: E731
    return (f"_ZN3sem13apply_band_kpILi{P}ELi{TXE}ELi{TYE}ELi{NS}E{b(full)}Li{cm}E{b(grad)}EEvPKdS2_S2_"
            "iiiiiiiiNS_8BandArgsE")


def compile_asm(out):
    src = open(os.path.join(ROOT, "sem_amd", "csrc", "apply_band.hip")).read()
    src = re.sub(r"SEM_BCASE\(1\) SEM_BCASE\(2\) SEM_BCASE\(3\) SEM_BCASE\(4\) SEM_BCASE\(5\) SEM_BCASE\(6\) "
                 r"SEM_BCASE\(7\) SEM_BCASE\(8\)", "SEM_BCASE(8)", src)
    src = re.sub(r"^ *SEM_BCASE\(9\).*SEM_BCASE\(16\)$", "", src, flags=re.M)
    d = os.path.join(ROOT, "sem_amd", ".isa_budget")
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, "apply_band_p8.hip")
    with open(p, "w") as f:
        f.write(src)
    for h in ("apply_common.h", "gll_consts.h", "sem_internal.h"):
        with open(os.path.join(ROOT, "sem_amd", "csrc", h)) as fi, open(os.path.join(d, h), "w") as fo:
            fo.write(fi.read())
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I",
                    os.path.join(ROOT, "include"), "-DSEM_DIAGNOSTICS=0", "-mllvm", "-amdgpu-kernarg-preload-count=14",
                    "--cuda-device-only", "-S", "-o", out, p], check=True, stderr=subprocess.DEVNULL)
    for fn in os.listdir(d):
        os.remove(os.path.join(d, fn))
    os.rmdir(d)


def category(op):
    if op.startswith("v_") and "f64" in op:
        if "fma" in op or "fmac" in op:
            return "VALU fp64 fma"
        return "VALU fp64 add/mul"
    if op.startswith("v_cmp") or op.startswith("v_cndmask"):
        return "VALU cmp/select"
    if op.startswith("v_"):
        return "VALU int/move"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "SMEM"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "SALU branch"
    if op.startswith("s_mov") or op.startswith("s_movk"):
        return "SALU move"
    if op.startswith("s_"):
        return "SALU other"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith("buffer_") or op.startswith("global_"):
        return "VMEM"
    return None


def budget(asm, name):
    lines = open(asm).read().split("\n")
    st = [i for i, l in enumerate(lines) if l.startswith(name + ":")][0]
    en = st
    while not lines[en].startswith(".Lfunc_end"):
        en += 1
    body = lines[st:en]
    bars = [i for i, l in enumerate(body) if l.strip().startswith("s_barrier")]
    cuts = [("prologue (tile map, staging loads -> LDS, pointwise loads)", 0, bars[0]),
            ("roles (X and Y contractions; a wave runs one of the role paths)", bars[0], bars[-1]),
            ("epilogue (X + Y + u, v terms, Dirichlet path, stores)", bars[-1], len(body))]
    out = []
    for label, a, b in cuts:
        c = collections.Counter()
        for l in body[a:b]:
            t = l.strip()
            if not t or t.startswith(";") or t.endswith(":") or t.startswith("."):
                continue
            k = category(t.split()[0])
            if k:
                c[k] += 1
        out.append((label, c))
    return out


def eo_plan_ops(P=8, NS=2, grad=True):
    """fp64 operations per element line of rows in the even-odd band plan (both K and G rows)."""
    H = (P + 1) // 2
    row0 = (2 * P if grad else P) + 2 * P + 2          # K, G FMAs; t[P+m] +- t[P-m]; the fold multiplies
    pair = (4 * H if grad else 2 * H) + (2 if P % 2 == 0 else 0) * (2 if grad else 1) + 4
    centre = (2 * H + 2) if P % 2 == 0 else 0
    eo = 2 * H
    npairs = (P - 1) // 2
    per_element_line = row0 + npairs * pair + centre + eo * (NS)     # e/o formed once per split that needs it
    return per_element_line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default="")
    ap.add_argument("--cm", type=int, default=0)
    ap.add_argument("--grad", type=int, default=1)
    a = ap.parse_args()
    asm = a.asm or os.path.join(tempfile.gettempdir(), "apply_band_p8.s")
    if not a.asm:
        compile_asm(asm)
    name = mangle(8, 1, 8, 2, False, a.cm, bool(a.grad))
    total = collections.Counter()
    for label, c in budget(asm, name):
        total.update(c)
        valu = sum(v for k, v in c.items() if k.startswith("VALU"))
        salu = sum(v for k, v in c.items() if k.startswith("SALU"))
        print(f"{label}: VALU {valu}, SALU {salu}, " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))
    per_line = eo_plan_ops(8, 2, bool(a.grad))
    # a tile: 8 lines x 64 columns = 512 nodes; X: 64 columns x one element line of rows; Y: 8 lines x 8 elements
    tile = 2 * 64 * per_line           # X (64 lanes) and Y (64 lanes) each carry one element line of rows
    print(f"even-odd plan: {per_line} fp64 ops per element line of rows (both directions' K{'+G' if a.grad else ''});"
          f" per tile of 512 nodes {tile} lane-ops = {tile / 512:.1f} per node = {tile / 64 / 4:.0f} VALU instructions"
          f" per wave (4 waves) -- the epilogue's combination adds ~4 per node")
    print("static totals: " + ", ".join(f"{k} {v}" for k, v in sorted(total.items())))


if __name__ == "__main__":
    sys.exit(main())
