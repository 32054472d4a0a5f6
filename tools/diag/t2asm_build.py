"""Diagnostic build only: reassemble the round-2 EvalMultCore kernel that
returned non-canonical words from the compiler output
kept from that build, plus patched variants, as code objects for
tensor2_asm_diag.hip.

The round-2 source was never committed, but `make asm` had written its ISA to
upmem--openfhe_amd/lib/ofhe_hip.s one minute before the failing run
(gpurun_out/dbg3.log): the kernel there has the grid-stride signature
k_tensor2(const TowerConst*, c0, c1, d0, d1, o0, o1, o2, u64 npairs, u32
log_n, u32 towers).  This script copies that kernel's text, descriptor and
metadata into t2_orig.s (committed, so the experiment does not depend on the
untracked build output) and writes the variants:

  orig      the compiler's code, unchanged
  nop       s_nop 4 before every SALU instruction that writes or reads the
            exec-save pair s[28:29] (s_*_saveexec_b64, s_xor_b64 / s_or_b64
            exec), i.e. wait states between the VALU carry-out writes of
            v_mad_u64_u32 ... s[28:29] and the SALU exec save / restore
  carry     the v_mad_u64_u32 carry-out pair renamed s[28:29] -> s[30:31]
            (next_free_sgpr raised), so the VALU never writes the SGPR pair the
            exec save lives in
  endwait   s_waitcnt vmcnt(0) before s_endpgm (stores drained before the
            wave's registers are released)
  zero      every VGPR v1..v55 zeroed at entry (reads of uninitialised
            registers would then see 0 in every wave)
  execnop   s_nop 4 after every SALU write of exec, before the next VALU
  nobranch  the ten exec-masked if/else blocks of the Barrett shift select
            (`s >= 64 ? ...`, taken the same way by every lane: nshift + 7 =
            65) replaced by their else bodies alone: no exec writes, no
            blocks executed under EXEC = 0
  vnop      s_nop 1 after every VALU instruction (two wait states between any
            VALU result and its next reader)
  rcpnop    s_nop 4 after the one transcendental instruction (v_rcp_iflag_f32,
            the reciprocal of `towers` for row % towers), before its consumer
  allnop    s_nop 4 after EVERY instruction of the kernel (five wait states
            everywhere: no intra-wave pipeline hazard survives this)
  nont      the loads and stores without the non-temporal hint (`off nt` ->
            `off`)
  vmwait    s_waitcnt vmcnt(0) after every global load (each load completes
            before the next instruction issues)
  dump      out0's store replaced by the lane's tower constants as the kernel
            holds them at the end: q (v[24:25]) in word 2i, nshift (v51) in
            the low half of word 2i + 1 -- checked against the table per
            element, next to that element's out2
  vgpr64    the unchanged code with its VGPR allocation raised from 56 to 64
            (next_free_vgpr / accum_offset / metadata only)
  vgpr48x   every wave's allocation 56 -> 72 (above 64: 7 waves per SIMD)
  vgprN     the same with the allocation raised to N = 80, 88, ..., 128
            (round 4: the sweep of every granule up to 128, 4+ waves per SIMD,
            so two or more 256-thread workgroups share each CU)
  dumpin    out0 receives the c1 pair as loaded (v[14:17], stored right after
            the first s_waitcnt that covers its load, through v[56:57]) and
            keeps nothing else: the kernel's own view of its inputs

  python tools/diag/t2asm_build.py [path/to/ofhe_hip.s]
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
KNAME = "_ZN4ofhe9k_tensor2ILi0EEEvPKNS_10TowerConstEPKmS5_S5_S5_PmS6_S6_mjj"
CLANG = "/opt/rocm/llvm/bin/clang"
LLD = "/opt/rocm/llvm/bin/ld.lld"


def extract(src):
    lines = open(src).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("\t.section\t.text." + KNAME))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith("\t.set " + KNAME + ".has_indirect_call"))
    text = lines[start:end + 1]
    md0 = next(i for i, l in enumerate(lines) if l.strip() == ".amdgpu_metadata")
    # the kernel's entry: from its "- .agpr_count" line to the next one
    name_at = next(i for i in range(md0, len(lines)) if lines[i].strip() == ".name:           " + KNAME)
    e0 = max(i for i in range(md0, name_at) if lines[i].startswith("  - .agpr_count"))
    e1 = next(i for i in range(name_at, len(lines)) if lines[i].startswith("  - ") or lines[i].startswith("amdhsa.target"))
    entry = lines[e0:e1]
    out = ['\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', "\t.amdhsa_code_object_version 6"] + text
    out += ["\t.amdgpu_metadata", "---", "amdhsa.kernels:"] + entry
    out += ["amdhsa.target:   amdgcn-amd-amdhsa--gfx950", "amdhsa.version:", "  - 1", "  - 2", "...", "",
            "\t.end_amdgpu_metadata", ""]
    return "\n".join(out)


THEN_BLOCKS = {"%%bb.%d:" % k for k in (4, 8, 12, 16, 20, 24, 28, 32)}


def nobranch(text):
    out, skip = [], False
    for l in text.split("\n"):
        s = l.strip()
        if s.startswith("; %bb.") or s.startswith(".LBB"):
            skip = s.split()[1] in THEN_BLOCKS if s.startswith(";") else False
            out.append(l)
            continue
        if skip and not s.startswith(";"):
            continue
        if re.match(r"s_\w+_saveexec_b64 s\[28:29\]", s) or s in (
                "s_xor_b64 s[28:29], exec, s[28:29]", "s_xor_b64 exec, exec, s[28:29]",
                "s_or_b64 exec, exec, s[28:29]", "s_cbranch_execz .LBB66_2"):
            continue
        out.append(l)
    return "\n".join(out)


def variant(text, kind):
    if kind == "orig":
        return text
    if kind == "nobranch":
        return nobranch(text)
    if kind == "nont":
        return text.replace(", off nt", ", off")
    if kind in ("vgpr64", "vgpr48x") or re.fullmatch(r"vgpr\d+", kind):
        n = 64 if kind == "vgpr64" else 72 if kind == "vgpr48x" else int(kind[4:])
        text = text.replace(".amdhsa_next_free_vgpr 56", ".amdhsa_next_free_vgpr %d" % n)
        text = text.replace(".amdhsa_accum_offset 56", ".amdhsa_accum_offset %d" % n)
        return re.sub(r"(\.vgpr_count:\s+)56", r"\g<1>%d" % n, text)
    if kind == "dumpin":
        old = "\tglobal_store_dwordx4 v[2:3], v[6:9], off nt"
        assert text.count(old) == 1
        text = text.replace(old, "")
        w = "\ts_waitcnt vmcnt(5)"
        assert text.count(w) == 1
        text = text.replace(w, w + "\n\tv_lshl_add_u64 v[56:57], s[12:13], 0, v[20:21]\n"
                                   "\tglobal_store_dwordx4 v[56:57], v[14:17], off")
        text = text.replace(".amdhsa_next_free_vgpr 56", ".amdhsa_next_free_vgpr 58")
        text = text.replace(".amdhsa_accum_offset 56", ".amdhsa_accum_offset 60")
        text = re.sub(r"(\.vgpr_count:\s+)56", r"\g<1>58", text)
        return text
    if kind == "dump":
        old = "\tglobal_store_dwordx4 v[2:3], v[6:9], off nt"
        assert text.count(old) == 1
        return text.replace(old, "\tglobal_store_dwordx2 v[2:3], v[24:25], off\n"
                                 "\tglobal_store_dword v[2:3], v51, off offset:8")
    out = []
    lines = text.split("\n")
    for i, l in enumerate(lines):
        s = l.strip()
        if kind == "nop" and (re.match(r"s_(and|or|andn2)_saveexec_b64 s\[28:29\]", s) or
                              re.match(r"s_(xor|or)_b64 (exec|s\[28:29\]), exec, s\[28:29\]", s)):
            out.append("\ts_nop 4")
        if kind == "carry" and s.startswith("v_mad_u64_u32") and "s[28:29]" in s:
            l = l.replace("s[28:29]", "s[30:31]")
        if kind == "carry":
            l = l.replace(".amdhsa_next_free_sgpr 30", ".amdhsa_next_free_sgpr 34")
            l = l.replace("numbered_sgpr, 30", "numbered_sgpr, 34")
            l = re.sub(r"(\.sgpr_count:\s+)(\d+)", lambda m: m.group(1) + str(max(int(m.group(2)), 40)), l)
        if kind == "endwait" and s == "s_endpgm":
            out.append("\ts_waitcnt vmcnt(0)")
        out.append(l)
        if kind == "zero" and s == "; %bb.0:":
            out += ["\tv_mov_b32_e32 v%d, 0" % k for k in range(1, 56)]
        if kind == "execnop" and (re.match(r"s_\w+_saveexec_b64", s) or re.match(r"s_\w+_b64 exec,", s)):
            out.append("\ts_nop 4")
        if kind == "vnop" and s.startswith("v_"):
            out.append("\ts_nop 1")
        if kind == "rcpnop" and s.startswith("v_rcp_iflag_f32"):
            out.append("\ts_nop 4")
        if kind == "allnop" and re.match(r"^[vs]_", s) and not s.startswith(("s_endpgm", "s_cbranch", "s_branch")):
            out.append("\ts_nop 4")
        if kind == "vmwait" and s.startswith("global_load"):
            out.append("\ts_waitcnt vmcnt(0)")
    return "\n".join(out)


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else None
    orig = os.path.join(HERE, "t2_orig.s.txt")
    if src:
        open(orig, "w").write(extract(src))
    text = open(orig).read()
    kinds = ["orig", "nop", "carry", "endwait", "zero", "execnop", "nobranch", "vnop", "rcpnop", "allnop", "nont",
             "vmwait", "dump", "dumpin", "vgpr64", "vgpr48x"]
    # round 4: the same machine code at every allocation from 64
    # to 128 VGPRs (granule 8), each run with two or more workgroups per CU
    kinds += ["vgpr%d" % n for n in range(80, 129, 8)]
    if os.environ.get("T2_KINDS"):
        kinds = os.environ["T2_KINDS"].split(",")
    for kind in kinds:
        s = os.path.join(HERE, f"t2_{kind}_gen.s")
        o = os.path.join(HERE, f"t2_{kind}.o")
        co = os.path.join(HERE, f"t2_{kind}.hsaco")
        open(s, "w").write(variant(text, kind))
        subprocess.check_call([CLANG, "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", s, "-o", o])
        subprocess.check_call([LLD, "-shared", o, "-o", co])
        os.remove(o)
        os.remove(s)
        print("built", co)


if __name__ == "__main__":
    main()
