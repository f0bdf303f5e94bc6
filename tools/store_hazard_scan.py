#!/usr/bin/env python3
"""List the vector stores of more than 8 bytes whose data VGPRs a VALU
instruction overwrites too soon after the store (DESIGN §4 "A store-data
hazard").  Measured on gfx950 (tools/ubench/store_hazard.hip): a 12- or 16-B
buffer store with an SGPR soffset needs 1 wait state before a VALU write of
its data VGPRs, with a constant soffset -- or a global store -- 2; LLVM's
hazard recognizer gives 0 and 1.  8-B stores need none.

    python3 tools/store_hazard_scan.py [--lib libsurfhip.so | file.s ...]

Default: the device code objects inside cuda-surf_amd/libsurfhip.so
(llvm-objdump --offloading, then -d).  .s files (hipcc --cuda-device-only
-S) are read as they are.  Wait states: one per instruction between the store
and the overwrite, s_nop k counting k + 1; branches are followed (both ways
for a conditional one).  Exit status 1 if any store violates the measured
rule.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import shutil
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-surf_amd")

STORE = re.compile(r"\s+(buffer|global|flat)_store_dwordx([34])\s+(?:v\[\d+:\d+\],\s*)?v\[(\d+):(\d+)\]")
BUF = re.compile(r"\s+buffer_store_dwordx[34]\s+v\[(\d+):(\d+)\],\s*\S+,\s*\S+,\s*([^\s,]+)")
GLB = re.compile(r"\s+(?:global|flat)_store_dwordx[34]\s+\S+,\s*v\[(\d+):(\d+)\]")
VALU = re.compile(r"\s+(v_\w+)\s+(?:v\[(\d+):(\d+)\]|v(\d+))\b")
NOP = re.compile(r"\s+s_nop\s+(\d+)")
FUNC = re.compile(r"^(?:[0-9a-f]+ <(\S+)>|(_Z\S+|\w+)):\s*(;.*)?$")


OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def disassemble_lib(lib: str, tmp: str | None = None) -> list[str]:
    """The gfx950 code objects bundled in a HIP shared library, disassembled
    into `tmp` (a new temporary directory when None; llvm-objdump extracts
    the bundles next to its input: work on a copy)."""
    tmp = tmp or tempfile.mkdtemp(prefix="hzscan")
    cp = os.path.join(tmp, "lib.so")
    shutil.copyfile(lib, cp)
    subprocess.run([OBJDUMP, "--offloading", cp], cwd=tmp, check=True, capture_output=True)
    out = []
    for name in sorted(os.listdir(tmp)):
        if "gfx950" in name:
            dst = os.path.join(tmp, name + ".dis")
            with open(dst, "w") as fh:
                subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", os.path.join(tmp, name)], stdout=fh, check=True)
            out.append(dst)
    return out


def need(soff: str) -> int:
    """wait states a wide store needs before its data VGPRs are rewritten"""
    return 1 if re.match(r"^(s\d+|vcc_\w+|m0|ttmp\d+)$", soff) else 2


ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<(\S+)\+0x([0-9a-f]+)>")
HEADER = re.compile(r"^([0-9a-f]+) <(\S+)>:")


def _index(lines):
    """label / address -> line index, for following branches"""
    labels, addr, base = {}, {}, {}
    for i, line in enumerate(lines):
        m = HEADER.match(line)
        if m:
            base[m.group(2)] = int(m.group(1), 16)
            continue
        if line.startswith(".L") and line.rstrip().endswith(":") or re.match(r"^\.LBB\S+:", line):
            labels[line.split(":")[0].strip()] = i
        a = ADDR.search(line)
        if a:
            addr[int(a.group(1), 16)] = i
    return labels, addr, base


def _targets(s, labels, addr, base):
    """line indices a branch instruction may continue at (besides falling
    through for a conditional one)"""
    t = TARGET.search(s)
    if t and t.group(1) in base:
        i = addr.get(base[t.group(1)] + int(t.group(2), 16))
        return [i] if i is not None else []
    parts = s.split()
    if len(parts) > 1 and parts[1] in labels:
        return [labels[parts[1]]]
    return []


def scan(path: str, within: int | None):
    lines = open(path).read().split("\n")
    labels, addr, base = _index(lines)
    cur = None
    hits = {}
    counts = {}

    def walk(j, ws, lim, lo, hi, depth):
        """first VALU write of v[lo:hi] at <= lim wait states from line j
        on (branches followed, conditional ones both ways), or None"""
        while j < len(lines) and depth < 8:
            t = lines[j].split("//")[0]
            s = t.strip()
            j += 1
            if not s or s.startswith(";") or s.startswith(".") and not s.endswith(":"):
                continue
            if re.match(r"^\S+:", t) or HEADER.match(lines[j - 1]):
                continue
            if s.startswith(("s_setpc", "s_endpgm", "s_trap")):
                return None
            if s.startswith("s_branch") or s.startswith("s_cbranch"):
                ws += 1
                if ws > lim:
                    return None
                for tj in _targets(lines[j - 1], labels, addr, base):
                    h = walk(tj, ws, lim, lo, hi, depth + 1)
                    if h:
                        return h
                if s.startswith("s_branch"):
                    return None
                continue
            n = NOP.match(t)
            if n:
                ws += int(n.group(1)) + 1
                if ws > lim:
                    return None
                continue
            v = VALU.match(t)
            if v and not v.group(1).startswith(("v_cmp", "v_readlane", "v_readfirstlane", "v_cmpx")):
                a = int(v.group(2) or v.group(4))
                z = int(v.group(3) or v.group(4))
                if not (z < lo or a > hi):
                    return (j, ws, s.split()[0])
            ws += 1
            if ws > lim:
                return None
        return None

    for i, line in enumerate(lines):
        m = FUNC.match(line)
        if m and not line.startswith("."):
            cur = m.group(1) or m.group(2)
            continue
        b = BUF.match(line)
        g = GLB.match(line) if not b else None
        if not (b or g) or cur is None:
            continue
        lo, hi = (int(b.group(1)), int(b.group(2))) if b else (int(g.group(1)), int(g.group(2)))
        soff = b.group(3) if b else "-"
        c = counts.setdefault(cur, [0, 0])
        c[0] += 1
        lim = need(soff) - 1 if within is None else within
        h = walk(i + 1, 0, lim, lo, hi, 0)
        if h:
            c[1] += 1
            hits.setdefault(cur, []).append((h[0], h[1], soff, h[2]))
    return counts, hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--within", type=int, default=None,
                    help="report overwrites at <= this many wait states (default: the measured rule)")
    ap.add_argument("--lib", default=os.path.join(PKG, "libsurfhip.so"))
    ap.add_argument("files", nargs="*")
    a = ap.parse_args()
    files = a.files or disassemble_lib(a.lib)
    total = 0
    for f in files:
        counts, hits = scan(f, a.within)
        for k, (ns, nh) in counts.items():
            if nh:
                total += nh
                ws = sorted({h[1] for h in hits[k]})
                soffs = sorted({h[2] for h in hits[k]})
                print(f"{os.path.basename(f)}: {k[:90]}: {nh} of {ns} wide stores overwritten at wait states {ws} "
                      f"(soffset {soffs})")
    rule = "the measured rule (SGPR soffset: < 1, otherwise < 2)" if a.within is None else f"<= {a.within}"
    print(f"{total} wide stores with a VALU overwrite of their data at {rule} wait states")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
