"""List every transcendental VALU instruction (v_rcp*, v_rsq*, v_sqrt*, v_exp*,
v_log*, v_sin*, v_cos*) in gfx950 assembly and the number of instructions
between it and the first later instruction that reads its result, per kernel
(diagnostic for the round-2 EvalMultCore failure).

  python tools/diag/trans_gaps.py file.s [...]
"""
import re
import sys

TRANS = re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)\w*")


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


for path in sys.argv[1:]:
    kern, lines = None, []
    out = {}
    for raw in open(path):
        s = raw.strip()
        m = re.match(r"^(_Z\w+):", raw)
        if m:
            kern, lines = m.group(1), []
            continue
        if not kern or not s or s.startswith((";", ".")):
            continue
        lines.append(s.split(";")[0].strip())
        if s.startswith("s_endpgm"):
            for i, l in enumerate(lines):
                if TRANS.match(l):
                    dst = regs(l.split(None, 1)[1].split(",")[0].strip())
                    gap = None
                    for j in range(i + 1, min(i + 40, len(lines))):
                        ops = lines[j].split(None, 1)
                        if len(ops) < 2:
                            continue
                        srcs = set()
                        for o in ops[1].split(",")[1:]:
                            srcs |= regs(o.strip())
                        if dst & srcs:
                            gap = j - i - 1
                            nops = sum(int(x.split()[1]) + 1 if len(x.split()) > 1 else 1
                                       for x in lines[i + 1:j] if x.startswith("s_nop"))
                            out.setdefault(kern, []).append((l.split()[0], gap, nops, lines[i + 1:j + 1]))
                            break
            kern = None
    for k, v in out.items():
        print(f"{path}: {k[:90]}")
        for ins, gap, nops, seq in v:
            print(f"    {ins}: {gap} instruction(s) before the consumer ({nops} s_nop wait states): "
                  + " | ".join(x.split()[0] for x in seq))
