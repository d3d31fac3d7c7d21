"""Static check of the LDS ring-slot invariant in the shipped gfx950 code (no GPU needed).

The round-3 race (fixed in 890d20b): in the LDS-DMA conv kernels a ring slot is released by an s_barrier, after which
another wave's `buffer_load_dwordx4 ... lds` refills it.  The DMA writes LDS through the vector-memory path, so it can
overtake a `ds_read` that a wave issued before the barrier but has not completed — unless every wave waits for its
own LDS reads (`s_waitcnt lgkmcnt(0)`) before the barrier.  This checker disassembles the library's code objects and,
in every kernel that issues LDS-DMA loads, runs a forward dataflow over the control-flow graph: state "a ds_read is
outstanding" is set by any ds_read*/ds_load* and cleared by an s_waitcnt whose lgkmcnt is 0; an s_barrier reached
with the state set on any path, from which an LDS-DMA load is reachable before the next s_barrier, is a violation.

    python tools/lds_barrier_check.py [path/to/libvmatting.so]     # prints violations, exit 1 if any
"""

import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:\s*$")
_INST = re.compile(r"^\s+([a-z_0-9]+)([^/]*)//\s*([0-9A-F]+):")
_TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>\s*$")


def disassemble(lib):
    """Extract every gfx950 code object of ``lib`` (a fat host binary) and return their disassembly text."""
    out = []
    with tempfile.TemporaryDirectory() as td:
        so = os.path.join(td, os.path.basename(lib))
        shutil.copy(lib, so)  # llvm-objdump --offloading writes the bundles next to its input
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], check=True, capture_output=True)
        for f in sorted(os.listdir(td)):
            if "amdgcn" in f and "gfx950" in f:
                r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", os.path.join(td, f)],
                                   check=True, capture_output=True, text=True)
                out.append(r.stdout)
    return out


def functions(text):
    """-> {name: (start address, [(addr, mnemonic, operands, line)])}"""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = m.group(2)
            funcs[cur] = (int(m.group(1), 16), [])
            continue
        m = _INST.match(line)
        if m and cur is not None:
            funcs[cur][1].append((int(m.group(3), 16), m.group(1), m.group(2).strip(), line))
    return funcs


def _clears(mn, ops):
    if mn == "s_waitcnt":
        m = re.search(r"lgkmcnt\((\d+)\)", ops)
        return m is not None and int(m.group(1)) == 0
    if mn == "s_waitcnt_lgkmcnt":
        return ops.replace(" ", "").endswith(",0x0") or ops.replace(" ", "").endswith(",0")
    return False


def _sets(mn):
    return mn.startswith("ds_read") or mn.startswith("ds_load")


def check_function(name, start, insts):
    """Violations [(name, addr, line)] of one kernel (empty if it issues no LDS-DMA load)."""
    if not any(mn.startswith(("buffer_load", "global_load")) and re.search(r"\blds\b", ops) for _, mn, ops, _ in insts):
        return []
    index = {a: i for i, (a, _, _, _) in enumerate(insts)}
    succ = []
    for i, (a, mn, ops, line) in enumerate(insts):
        s = []
        tgt = None
        m = _TARGET.search(line)
        if m and m.group(1) == name and (mn.startswith("s_branch") or mn.startswith("s_cbranch")):
            tgt = index.get(start + int(m.group(2), 16))
        if mn == "s_branch":
            s = [tgt] if tgt is not None else []
        elif mn in ("s_endpgm", "s_setpc_b64"):
            s = []
        else:
            if i + 1 < len(insts):
                s.append(i + 1)
            if mn.startswith("s_cbranch") and tgt is not None:
                s.append(tgt)
        succ.append(s)
    pending_in = [False] * len(insts)
    reached = [False] * len(insts)
    reached[0] = True
    work = [0]
    while work:  # forward dataflow, OR at joins
        i = work.pop()
        _, mn, ops, _ = insts[i]
        st = pending_in[i]
        if _sets(mn):
            st = True
        elif _clears(mn, ops):
            st = False
        for j in succ[i]:
            if not reached[j] or (st and not pending_in[j]):
                reached[j] = True
                pending_in[j] = pending_in[j] or st
                work.append(j)
    # a barrier with an outstanding read is a race only if an LDS-DMA load can follow it before the next barrier
    # (LDS reads and ds_writes of different waves are served in issue order; the DMA path is not)
    is_dma = [mn.startswith(("buffer_load", "global_load")) and re.search(r"\blds\b", ops) is not None
              for _, mn, ops, _ in insts]

    def dma_follows(i0):
        seen, stack = set(), list(succ[i0])
        while stack:
            j = stack.pop()
            if j in seen:
                continue
            seen.add(j)
            if is_dma[j]:
                return True
            if insts[j][1] != "s_barrier":
                stack.extend(succ[j])
        return False

    return [(name, a, line.strip()) for i, (a, mn, _, line) in enumerate(insts)
            if mn == "s_barrier" and reached[i] and pending_in[i] and dma_follows(i)]


def check_library(lib):
    bad, kernels = [], 0
    for text in disassemble(lib):
        for name, (start, insts) in functions(text).items():
            v = check_function(name, start, insts)
            if any(mn.startswith(("buffer_load", "global_load")) and re.search(r"\blds\b", ops)
                   for _, mn, ops, _ in insts):
                kernels += 1
            bad += v
    return bad, kernels


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "video-matting_amd", "vmatting", "libvmatting.so")
    bad, kernels = check_library(lib)
    print("%d kernels with LDS-DMA loads checked, %d barrier(s) with an outstanding ds_read" % (kernels, len(bad)))
    for name, a, line in bad:
        print("  %s @%x: %s" % (name, a, line))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
