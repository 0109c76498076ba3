"""Instruction census of K1's per-pixel loop, from the compiled gfx950 code.

    python tools/k1_census.py [--out profiles/r05/k1_census.txt]

Compiles photohive_dsp_amd/csrc/k1.hip to device assembly with the library's
own flags (Makefile HIPFLAGS + K1FLAGS), finds every k_k1t instance, takes the
innermost loop holding the pixel loads (the pixel loop: one 12-byte load =
4 RGB8 pixels per thread and iteration) and counts its
instructions by class.  Runs anywhere hipcc does (no GPU)."""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "photohive_dsp_amd", "csrc", "k1.hip")
FLAGS = ["-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-munsafe-fp-atomics", "-mllvm", "-phi-node-folding-threshold=32", "-mllvm",
         "-two-entry-phi-node-folding-threshold=32", "--cuda-device-only", "-S"]


def classify(op):
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu/branch"
    if op.startswith("v_"):
        if "_f64" in op or op.startswith("v_fma_f64") or op.startswith("v_rcp_f64"):
            return "valu fp64"
        if op.startswith("v_mov") or op.startswith("v_accvgpr"):
            return "valu move"
        if op.startswith("v_cndmask"):
            return "valu select"
        if op.startswith("v_pk_"):
            return "valu packed"
        return "valu other"
    return "other"


def loops(lines):
    """(header label, body lines) of every loop: a label whose own name a later
    branch targets, body = the lines between them."""
    pos = {}
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            pos[m.group(1)] = i
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
        if m:
            t = m.group(1) or m.group(2)
            if t in pos and pos[t] < i:
                out.append((t, lines[pos[t]:i + 1]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--asm", default=None, help="an already compiled k1.s (e.g. an A/B build's flags)")
    a = ap.parse_args()
    if a.asm:
        text = open(a.asm).read().splitlines()
    else:
        with tempfile.TemporaryDirectory() as d:
            s = os.path.join(d, "k1.s")
            subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + ["-o", s, SRC], check=True)
            text = open(s).read().splitlines()
    # split by function
    funcs = collections.OrderedDict()
    cur = None
    for l in text:
        m = re.match(r"^(_Z\S*k_k1t\S*):", l)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur and l.startswith(".Lfunc_end"):
            cur = None
        if cur:
            funcs[cur].append(l.strip())
    rep = []
    demangle = {}
    if funcs:
        r = subprocess.run(["c++filt"] + list(funcs), capture_output=True, text=True)
        demangle = dict(zip(funcs, r.stdout.splitlines()))
    for f, body in funcs.items():
        lp = loops(body)
        if not lp:
            continue
        # the pixel loops: the innermost loops holding the 12-byte pixel load
        # (dwordx3): the per-pixel form (three LDS atomics per pixel, straight
        # line) and the cell-run form (atomics only when a thread's cell
        # changes, behind an exec-mask branch; chunks a block vote found flat)
        heads = {h for h, _ in lp}
        for hdr, b in lp:
            if any(x.endswith(":") and x[:-1] in heads and x[:-1] != hdr for x in
                   (y.split()[0] for y in b if y)):
                continue                                   # not innermost
            ins = [x for x in b if x and not x.startswith((".", ";")) and not x.endswith(":")]
            if not any("global_load_dwordx3" in x or "global_load_dwordx2" in x for x in ins):
                continue
            guarded = any(x.startswith("ds_add_u64") and any("s_cbranch_execz" in y for y in ins[max(0, i - 4):i])
                          for i, x in enumerate(ins))
            c = collections.Counter(classify(x.split()[0]) for x in ins)
            ops = collections.Counter(x.split()[0] for x in ins)
            form = "cell-run form" if guarded else "per-pixel form"
            rep.append(f"{demangle.get(f, f)}\n  {form}, loop {hdr}: {len(ins)} instructions per iteration "
                       f"(4 pixels per thread)")
            for k in ("valu fp64", "valu other", "valu packed", "valu move", "valu select", "lds", "vmem",
                      "salu/branch", "waitcnt", "other"):
                if c[k]:
                    rep.append(f"    {k:12s} {c[k]:4d}  ({c[k] / 4:.2f} per pixel)")
            nval = sum(v for k, v in c.items() if k.startswith("valu"))
            rep.append(f"    {'valu total':12s} {nval:4d}  ({nval / 4:.2f} per pixel)")
            rep.append("    top opcodes: " + ", ".join(f"{o} {n}" for o, n in ops.most_common(14)))
    txt = "\n".join(rep) + "\n"
    sys.stdout.write(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write("# tools/k1_census.py (compiled k1.hip, gfx950, library flags)\n" + txt)


if __name__ == "__main__":
    main()
