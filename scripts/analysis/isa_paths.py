"""Walk one path through a kernel's gfx950 ISA and count its instructions
(the ISA census of DESIGN.md §4, round 6).  Analysis only.

  python scripts/analysis/isa_paths.py KERN.s SYMBOL START STOP_LINE POLICY...

KERN.s: hipcc -S -gline-tables-only output.  The walk starts at label START
(.LBBx_y) or at the first instruction whose innermost lzma_device.h line is START and ends when it
reaches an instruction of STOP_LINE again (or after 2,000 instructions).  Each
conditional branch is resolved by POLICY entries LINE=t|n (taken / not taken)
keyed on a lzma_device.h line of the branch's inline chain (the innermost one
with an entry wins); a branch with no entry is not taken.  Prints the path and its counts by class.
"""
import re
import sys
from collections import Counter

LOC = re.compile(r"^\s*\.loc\s+\d+\s+(\d+)\s+\d+.*?;\s*(.*)$")


def load(path, sym):
    ins, lab = [], {}
    cur = None
    on = False
    for raw in open(path):
        if not on:
            if raw.startswith("_Z") and sym in raw.split(":")[0]:
                on = True
            continue
        if raw.startswith(".Lfunc_end"):
            break
        m = LOC.match(raw)
        if m:
            parts = re.findall(r"([\w./-]+\.(?:h|hip)):(\d+)", m.group(2))
            cur = [(p.rsplit("/", 1)[-1], int(n)) for p, n in parts]
            continue
        m = re.match(r"^(\.LBB\d+_\d+):", raw)
        if m:
            lab[m.group(1)] = len(ins)
            continue
        if raw.startswith("\t") and not raw.strip().startswith((".", ";")) and raw.strip():
            devs = [n for f, n in (cur or []) if f == "lzma_device.h"]
            ins.append((raw.strip().split(";")[0].strip(), devs[0] if devs else 0, devs))
    return ins, lab


def cls(op):
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait/nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "valu"


def walk(ins, lab, start, stop, policy, limit=2000):
    if isinstance(start, str):
        i = lab[start]  # a label
    else:
        i = next(k for k, (_, d, _c) in enumerate(ins) if d == start)
    path = []
    seen_start = False
    while len(path) < limit and i < len(ins):
        t, d, chain = ins[i]
        if d == stop and seen_start:
            break
        seen_start = True
        path.append((t, d))
        op = t.split()[0]
        if op == "s_branch":
            i = lab[t.split()[1]]
            continue
        if op.startswith("s_cbranch"):
            # the innermost line of the branch's inline chain with a policy
            dec = next((policy[c] for c in chain if c in policy), "n")
            if dec == "t":
                i = lab[t.split()[1]]
                continue
        i += 1
    return path


def main():
    path, sym = sys.argv[1], sys.argv[2]
    start = sys.argv[3] if sys.argv[3].startswith(".") else int(sys.argv[3])
    stop = int(sys.argv[4])
    policy = {}
    for a in sys.argv[5:]:
        k, v = a.split("=")
        policy[int(k)] = v
    ins, lab = load(path, sym)
    p = walk(ins, lab, start, stop, policy)
    for t, d in p:
        print(f"  {t:<60} ; device:{d}")
    c = Counter(cls(t.split()[0]) for t, _ in p)
    print(len(p), "instructions:", dict(c))


if __name__ == "__main__":
    main()
