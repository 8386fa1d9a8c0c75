"""Static instruction mix of one kernel in a hipcc --save-temps .s file: counts by class
(MFMA, packed / plain VALU by opcode, LDS, VMEM, SALU, waits).  Static counts only (the K
loops are fully unrolled, so for these kernels they track the dynamic counts closely).
    python tools/isa_mix.py <file.s> <kernel-symbol-substring> [--top N]"""
import re
import sys
from collections import Counter


def kernel_body(path, sub):
    lines = open(path).read().splitlines()
    out, on = [], False
    for ln in lines:
        if not on and re.match(r"^(_Z\S*):", ln) and sub in ln and "amdgpu" not in ln:
            on = True
            name = ln[:-1]
            continue
        if on:
            if ln.startswith(".Lfunc_end") or ln.strip().startswith(".size"):
                break
            out.append(ln.strip())
    return out


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    body = kernel_body(path, sub)
    ops = [l.split()[0] for l in body if l and not l.startswith((".", ";", "//")) and not l.endswith(":")]
    cls = Counter(classify(o) for o in ops)
    print(f"{sub}: {len(ops)} instructions:", dict(cls))
    valu = Counter(o for o in ops if classify(o) in ("valu", "valu_pk"))
    for o, c in valu.most_common(top):
        print(f"  {o:28s} {c}")


if __name__ == "__main__":
    main()
