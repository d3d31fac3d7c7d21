"""Static guard of the LDS ring-slot race fix (890d20b), no GPU involved.

tools/lds_barrier_check.py disassembles the shipped library's gfx950 code objects and, in every kernel that issues
LDS-DMA loads (`buffer_load_dwordx4 ... lds`), requires that no s_barrier is reached with a ds_read still outstanding
(no `s_waitcnt lgkmcnt(0)` since it, on any control-flow path) when an LDS-DMA load can follow that barrier before the
next one: the refill DMA of the released slot could otherwise overtake the read.  On the library built from
890d20b^ the checker reports 12 such barriers in 8 kernels (among them the 4 x 32 folded-upconv instantiation
conv3x3_patch<64, 4, 1, 2, 4, 2, 9, false, 0, false, 3, true> whose race the world-2 test caught); on HEAD none."""

import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "video-matting_amd", "vmatting", "libvmatting.so")
sys.path.insert(0, os.path.join(REPO, "tools"))


@pytest.mark.skipif(not os.path.exists(LIB) or shutil.which("llvm-objdump", path="/opt/rocm/lib/llvm/bin") is None,
                    reason="needs the built library and ROCm's llvm-objdump")
def test_no_lds_dma_barrier_with_outstanding_reads():
    import lds_barrier_check as chk
    bad, kernels = chk.check_library(LIB)
    assert kernels >= 20, "expected the LDS-DMA conv kernels in the shipped library, found %d" % kernels
    assert not bad, "\n".join("%s @%x" % (n, a) for n, a, _ in bad)
