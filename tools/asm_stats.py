#!/usr/bin/env python3
"""Static instruction histogram and VALU issue estimate per kernel.

usage: python tools/asm_stats.py [path.s] [name-substring] [coeffs-per-thread]

Input is `make -C upmem--openfhe_amd/csrc asm`.  Weights are the issue cost in
full-rate slots measured by tools/microbench/oprate2.hip on gfx950:
32-bit integer multiplies are quarter rate, 64-bit adds/compares half rate.
"""
import collections
import re
import sys

COST = {
    "v_mad_u64_u32": 4, "v_mul_lo_u32": 4, "v_mul_hi_u32": 4,
    "v_lshl_add_u64": 2, "v_cmp_le_u64_e32": 2, "v_cmp_gt_u64_e32": 2, "v_cmp_lt_u64_e32": 2,
    "v_cmp_ge_u64_e32": 2, "v_cmp_le_u64_e64": 2, "v_cmp_gt_u64_e64": 2, "v_lshlrev_b64": 2,
    "v_lshrrev_b64": 2, "v_mov_b64_e32": 1,
}

path = sys.argv[1] if len(sys.argv) > 1 else "upmem--openfhe_amd/lib/ofhe_hip.s"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_"
cpt = float(sys.argv[3]) if len(sys.argv) > 3 else 0
s = open(path).read()
for m in re.finditer(r'\n(_Z\w+):[^\n]*\n(.*?)\n\s*s_endpgm', s, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    ins = [l.split()[0] for l in body.split('\n') if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
    c = collections.Counter(ins)
    valu = sum(v * COST.get(k, 1) for k, v in c.items() if k.startswith("v_"))
    meta = re.search(r'\.name:\s+' + re.escape(name) + r'\s.*?\.vgpr_count:\s+(\d+)', s, re.S)
    extra = f" valu_slots={valu}" + (f" slots/coeff={valu / cpt:.1f}" if cpt else "")
    print(f"{name[:70]} total={len(ins)}{extra}")
    print("   ", ", ".join(f"{k}:{v}" for k, v in sorted(c.items(), key=lambda x: -x[1])[:30]))
