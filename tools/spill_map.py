#!/usr/bin/env python3
"""Where the register spills of the shortest-path kernels sit (CPU only).

Compiles shadow_amd/csrc/routes.hip for gfx950 to assembly with line tables (or
reads an existing .s given with --asm), and for each product kernel instance lists:
  * the compiler's resource usage (VGPRs, SGPRs, spills, scratch bytes per lane);
  * every loop of the function (a backward branch) with its scratch loads/stores
    and SGPR-spill lane moves (v_readlane / v_writelane), and the source lines
    it spans;
  * the hot loops named by their source line: the relaxation loop (phase 2 of a
    round), the predecessor pass loop and the epilogue's walk, with their counts.
usage: python tools/spill_map.py [--asm routes.s] [kernel-substring ...]
"""
import argparse
import collections
import hashlib
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "shadow_amd", "csrc", "routes.hip")
DEFAULT = ["k_routes_passILi16ELi1024ELi1E", "k_routes_ssspILi16ELi1024ELi1ELb0E", "k_routes_ssspILi16ELi1024ELi2ELb0E",
           "k_routes_passILi16ELi1024ELi2E"]


def compile_asm(out):
    sha = hashlib.sha256(open(SRC, "rb").read()).hexdigest()[:16]
    fast = ["-DSHDR_ANALYSIS"] if os.environ.get("SPILL_FAST") else []
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-unused-parameter",
           f'-DSHDR_SRC_SHA="{sha}"', "--cuda-device-only", "-gline-tables-only", "-S", SRC, "-o", out,
           "-Rpass-analysis=kernel-resource-usage"] + fast + os.environ.get("SPILL_DEFS", "").split()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-2000:])
    usage = collections.defaultdict(dict)
    name = None
    for l in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", l)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"remark: (.*?): (\d+) \[", l)
        if m and name:
            usage[name][m.group(1).strip()] = int(m.group(2))
    return usage


def source_markers():
    """(first, last) source lines of each hot loop's body: the loop reported is the
    innermost one holding instructions of both."""
    lines = open(SRC).read().split("\n")

    def at(text, after=0):
        return next(i for i, l in enumerate(lines, 1) if i > after and text in l)
    relax = at("for (int32_t k = 0; k < witers; ++k)")
    pred = at("for (int32_t k = 0; k < witers; ++k)", relax)
    walk = at("walk back to the source, recording the in-arcs")
    # lines that compile to instructions of their own (compares, counters, branches)
    return {"relaxation (phase 2)": (at("const bool act = du0 - off < thr;", relax), at("if (cnt >= kFlushAt)", relax)),
            "predecessor pass": (at("const bool fresh = (d0.w & 1) || (d1.w & 1);", pred),
                                 at("if (d0.w & 2) {  // last item of the vertex", pred)),
            "epilogue walk": (at("if (hc[c] < kStack) s_stack", walk), at("} else if (vc[c] == s) {", walk))}


def analyse(lines, fn):
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and fn in l.split(":")[0])
    name = lines[start].split(":")[0]
    end = start
    while not lines[end].startswith(".Lfunc_end"):
        end += 1
    cur, labels, ins = 0, {}, []
    for l in lines[start:end]:
        m = re.match(r"\s*\.loc\s+\d+\s+(\d+).*;\s*(\S+):\d+:\d+", l)
        if m:  # (lines of inlined HIP headers count as 0)
            cur = int(m.group(1)) if m.group(2).endswith("routes.hip") else 0
            continue
        if re.match(r"\s*\.loc\s", l):
            continue
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        s = l.strip()
        if not s or s[0] in ";." or s.startswith("//"):
            continue
        ins.append((s.split()[0], cur))
    loops = []
    # backward branches
    raw = [l.strip() for l in lines[start:end]]
    k = 0
    for l in raw:
        if not l or l[0] in ";." or l.startswith("//") or re.match(r"^\.LBB\S+:", l):
            continue
        op = l.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = l.split()[-1]
            if tgt in labels and labels[tgt] <= k:
                loops.append((labels[tgt], k))
        k += 1

    def count(a, b):
        c = collections.Counter()
        for op, _ in ins[a:b + 1]:
            if op.startswith("scratch_load"):
                c["scratch_load"] += 1
            elif op.startswith("scratch_store"):
                c["scratch_store"] += 1
            elif op.startswith("v_readlane"):
                c["v_readlane"] += 1
            elif op.startswith("v_writelane"):
                c["v_writelane"] += 1
        return c
    return name, ins, sorted(set(loops)), count


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("kernels", nargs="*")
    a = ap.parse_args()
    usage = {}
    asm = a.asm
    if not asm:
        asm = os.path.join(tempfile.mkdtemp(), "routes.s")
        print(f"# assembly: {asm}")
        usage = compile_asm(asm)
    lines = open(asm).read().split("\n")
    marks = source_markers()
    print(f"# routes.hip sha {hashlib.sha256(open(SRC, 'rb').read()).hexdigest()[:16]}; hot-loop source lines {marks}")
    for fn in a.kernels or DEFAULT:
        name, ins, loops, count = analyse(lines, fn)
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dem = dem.replace("(anonymous namespace)::", "").split("(")[0]
        u = usage.get(name, {})
        print(f"\n== {dem}: {len(ins)} instructions; " + ", ".join(f"{k} {v}" for k, v in u.items()))
        print(f"   whole function: {dict(count(0, len(ins) - 1))}")
        for what, (l0, l1) in marks.items():
            # the innermost loop whose instructions carry both marker lines
            cands = [(b - a, a, b) for a, b in loops
                     if any(ln == l0 for _, ln in ins[a:b + 1]) and any(ln == l1 for _, ln in ins[a:b + 1])]
            # one per inlined copy (k_routes_pass holds the half-width and the full-width body)
            inner = [(n, a0, b0) for n, a0, b0 in cands if not any(a <= a0 and b0 <= b and (a, b) != (a0, b0)
                                                                   for _, a, b in cands) or
                     not any(a0 <= a and b <= b0 and (a, b) != (a0, b0) for _, a, b in cands)]
            inner = [(n, a0, b0) for n, a0, b0 in cands
                     if not any(a0 <= a and b <= b0 and (a, b) != (a0, b0) for _, a, b in cands)]
            for _, a0, b0 in sorted(inner, key=lambda x: x[1]):
                lns = [ln for _, ln in ins[a0:b0 + 1] if ln]
                print(f"   {what:22s} loop of {b0 - a0 + 1:5d} instructions (src {min(lns)}-{max(lns)}): "
                      f"{dict(count(a0, b0)) or 'no scratch access, no SGPR lane move'}")
        print("   every loop with a scratch access (innermost first):")
        for a0, b0 in sorted(loops, key=lambda x: x[1] - x[0]):
            c = count(a0, b0)
            if c["scratch_load"] + c["scratch_store"] == 0:
                continue
            lns = [ln for _, ln in ins[a0:b0 + 1] if ln] or [0]
            top = collections.Counter(lns).most_common(2)
            print(f"     [{a0},{b0}] {b0 - a0 + 1:5d} instr, src {min(lns)}-{max(lns)} (mostly {top}): {dict(c)}")


if __name__ == "__main__":
    main()
