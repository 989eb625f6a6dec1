"""Instruction mix of a kernel's loops in an amdgcn .s dump (hipcc
--cuda-device-only -S): per loop (a label with a backward branch to it),
counts of MFMA, VALU (other v_*), LDS (ds_*), global/buffer, SALU, waits.
  python tools/isa_mix.py FILE.s SYMBOL_SUBSTRING"""
import re
import sys
from collections import Counter


def kernel_lines(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.split(";")[0].strip().endswith(":") and sym in l and l.startswith("_Z"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accvgpr"
    if op.startswith("v_exp") or op.startswith("v_log") or op.startswith("v_rcp"):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    labels = {}
    insts = []
    for l in lines:
        t = l.strip()
        if re.match(r"^\.LBB\w+:", t):
            labels[t[:-1]] = len(insts)
        elif t and not t.startswith((";", ".")) and not t.endswith(":"):
            insts.append(t.split(";")[0].strip())
    loops = []
    for i, ins in enumerate(insts):
        m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\w+)", ins)
        if m and m.group(2) in labels and labels[m.group(2)] <= i:
            loops.append((labels[m.group(2)], i))
    tot = Counter(classify(x.split()[0]) for x in insts)
    print("kernel", dict(tot), "total", len(insts))
    for a, b in loops:
        c = Counter(classify(x.split()[0]) for x in insts[a:b + 1])
        if c["mfma"]:
            v = c["valu"] + c["trans"] + c["accvgpr"]
            print(f"loop [{a},{b}] {dict(c)}  VALU/MFMA {v / c['mfma']:.2f}")
            ops = Counter(x.split()[0] for x in insts[a:b + 1] if classify(x.split()[0]) in ("valu", "trans"))
            print("   top VALU:", ops.most_common(18))


if __name__ == "__main__":
    main()


def pattern(path, sym, lo, hi):
    """Compact class string of instructions [lo, hi] of a kernel: M mfma, v valu,
    e transcendental, d lds, g vmem, s salu, w wait."""
    lines = kernel_lines(path, sym)
    insts = [t.strip().split(";")[0].strip() for t in lines
             if t.strip() and not t.strip().startswith((";", ".")) and not t.strip().endswith(":")]
    code = {"mfma": "M", "valu": "v", "trans": "e", "lds": "d", "vmem": "g", "salu": "s", "wait": "w",
            "accvgpr": "a", "other": "o"}
    return "".join(code[classify(x.split()[0])] for x in insts[lo:hi + 1])
