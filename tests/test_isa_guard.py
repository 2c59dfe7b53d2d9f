"""CPU: an ISA-level guard on the shipped library's code object (no GPU needed).

The C = 256 trunk's residual scratch goes through a buffer resource (tower_wide.h `ScrBuf`).  Round 4
found that a `buffer_store_dwordx4` whose soffset operand is an SGPR is emitted WITHOUT the store-data
wait state gfx950 needs (LLVM's store-data hazard check exempts MUBUF stores with an SGPR soffset; the
next VALU write of the data registers went out with the store: wrong outputs,
profiles/r04/c256_rsrc/probe_summary.txt), while the soffset-free form gets it.  The shipped kernels
therefore issue every buffer store with soffset 0 and the whole offset in the voffset.  A toolchain or
code change that brings the SGPR-soffset form back would otherwise be caught only by the GPU tower
tests; this test disassembles libspmcts.so's gfx950 code objects and fails on any such store.
"""
import glob
import os
import re
import shutil
import subprocess
import tempfile

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "self_play_reinforcement_learning_amd",
                   "libspmcts.so")


def _disassembly(so):
    d = tempfile.mkdtemp(prefix="spmcts_isa_")
    try:
        x = os.path.join(d, "x.so")
        shutil.copy(so, x)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", x], cwd=d, check=True, capture_output=True)
        cos = sorted(glob.glob(os.path.join(d, "x.so.*gfx950*")))
        assert cos, "no gfx950 code object in the library"
        return [subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", f], check=True, capture_output=True,
                               text=True).stdout for f in cos]
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _buffer_stores(text):
    """(kernel, mnemonic, soffset operand) of every MUBUF store."""
    out, kern = [], None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            kern = m.group(1)
            continue
        s = line.strip()
        if s.startswith("buffer_store_"):
            ins = s.split("//")[0].split()
            ops = " ".join(ins[1:]).split(",")
            out.append((kern, ins[0], ops[3].split()[0] if len(ops) > 3 else None))
    return out


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-objdump"), reason="ROCm llvm-objdump absent")
def test_no_sgpr_soffset_buffer_stores():
    assert os.path.exists(LIB), "build the library first (__graft_entry__.build())"
    stores = [s for t in _disassembly(LIB) for s in _buffer_stores(t)]
    assert stores, "expected the C = 256 trunk's residual-scratch buffer stores"
    assert any("k_tower_dyn" in (k or "") for k, _, _ in stores)
    bad = [s for s in stores if s[2] is None or re.fullmatch(r"s\d+|s\[\d+:\d+\]|m0|ttmp\d+", s[2])]
    assert not bad, f"{len(bad)} buffer stores with a register soffset (missing wait state on gfx950): {bad[:5]}"
