"""Every kernel of the shipped library allocates at least 64 VGPRs.

The round-2 EvalMultCore kernel (grid-stride k_tensor2) returned wrong words
whenever its 56-VGPR waves shared a CU with other workgroups; its unchanged
machine code with the allocation raised to 64 or 72 VGPRs is exact
(tools/diag/tensor2_asm_diag.hip, DESIGN.md "The round-2 EvalMultCore
failure").  csrc/arith.hpp's OFHE_VGPR_FLOOR() holds every kernel at >= 64.
This test reads the allocation each kernel's descriptor asks the hardware for
(COMPUTE_PGM_RSRC1.GRANULATED_WORKITEM_VGPR_COUNT, granule 8 on gfx950) from
the gfx950 code object inside the built library -- no GPU needed.
"""
import os
import struct

import pytest

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "upmem--openfhe_amd", "lib", "libofhe_hip.so")


def _sections(elf):
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    secs = []
    for i in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + i * shentsize)
        secs.append(dict(name=name, type=typ, addr=addr, off=off, size=size, link=link, entsize=entsize))
    strtab = secs[shstrndx]
    for s in secs:
        end = elf.index(b"\0", strtab["off"] + s["name"])
        s["name"] = elf[strtab["off"] + s["name"]:end].decode()
    return secs


def _section_bytes(elf, name):
    s = next(s for s in _sections(elf) if s["name"] == name)
    return elf[s["off"]:s["off"] + s["size"]]


def _gfx950_code_object(lib):
    fb = _section_bytes(lib, ".hip_fatbin")
    assert fb[:24] == b"__CLANG_OFFLOAD_BUNDLE__"
    n, = struct.unpack_from("<Q", fb, 24)
    p = 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", fb, p)
        p += 24
        triple = fb[p:p + tl].decode()
        p += tl
        if triple.endswith("gfx950"):
            return fb[off:off + size]
    raise AssertionError("no gfx950 code object in the library")


def kernel_vgpr_allocations(co):
    """{kernel symbol: VGPRs allocated per lane} from the kernel descriptors"""
    secs = _sections(co)
    symtab = next(s for s in secs if s["type"] == 2)  # SHT_SYMTAB
    strtab = secs[symtab["link"]]
    out = {}
    for k in range(symtab["size"] // symtab["entsize"]):
        name, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", co, symtab["off"] + k * symtab["entsize"])
        end = co.index(b"\0", strtab["off"] + name)
        sym = co[strtab["off"] + name:end].decode()
        if not sym.endswith(".kd"):
            continue
        sec = secs[shndx]
        kd = co[sec["off"] + value - sec["addr"]:][:64]
        rsrc1, = struct.unpack_from("<I", kd, 48)
        out[sym[:-3]] = ((rsrc1 & 0x3F) + 1) * 8
    return out


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_every_kernel_allocates_at_least_64_vgprs():
    lib = open(LIB, "rb").read()
    alloc = kernel_vgpr_allocations(_gfx950_code_object(lib))
    assert len(alloc) > 50, "kernel descriptors not found"
    assert any("k_tensor2" in k for k in alloc) and any("k_eltwise" in k for k in alloc)
    low = {k: v for k, v in alloc.items() if v < 64}
    assert not low, f"kernels below the 64-VGPR floor: {low}"
