"""Annotate a kernel's gfx950 ISA (hipcc -S -gline-tables-only) with its source.

  python scripts/analysis/isa_annotate.py KERN.s SYMBOL_SUBSTR [--lines]

Prints every instruction of the first function whose symbol contains
SYMBOL_SUBSTR, prefixed by its innermost lzma_device.h / lzma_lane.h line and the
chain of inlined call sites (innermost first), plus basic-block labels.  With
--lines: instruction counts per innermost source line instead (static census).
"""
import re
import sys
from collections import Counter

LOC = re.compile(r"^\s*\.loc\s+\d+\s+(\d+)\s+\d+.*?;\s*(.*)$")
INS = re.compile(r"^\s+([a-z_][a-z0-9_]*)(\s|$)")
LBL = re.compile(r"^(\.LBB\d+_\d+|\S+):")


def chain(comment):
    # "csrc/lzma_device.h:783:19 @[ csrc/lzma_device.h:811:41 @[ ... ] ]"
    parts = re.findall(r"([\w./-]+\.(?:h|hip)):(\d+)", comment)
    return [(p.rsplit("/", 1)[-1], int(n)) for p, n in parts]


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines_mode = "--lines" in sys.argv
    on = False
    cur = []
    cnt = Counter()
    with open(path) as f:
        for raw in f:
            if not on:
                if raw.startswith("_Z") and sym in raw.split(":")[0]:
                    on = True
                    print("==", raw.split(":")[0])
                continue
            if raw.startswith(".Lfunc_end"):
                break
            m = LOC.match(raw)
            if m:
                cur = chain(m.group(2))
                continue
            m = LBL.match(raw)
            if m and not raw.startswith("\t"):
                if not lines_mode:
                    print(m.group(1) + ":" + (raw.split(";", 1)[1].rstrip() if ";" in raw else ""))
                continue
            m = INS.match(raw)
            if not m or raw.strip().startswith("."):
                continue
            op = m.group(1)
            src = " < ".join(f"{f.split('.')[0][-6:]}:{n}" for f, n in cur[:4])
            if lines_mode:
                key = f"{cur[0][0]}:{cur[0][1]}" if cur else "?"
                cnt[key] += 1
            else:
                print(f"  {raw.strip().split(';')[0]:<60} ; {src}")
    if lines_mode:
        for k, v in sorted(cnt.items(), key=lambda kv: -kv[1]):
            print(f"{v:6d} {k}")


if __name__ == "__main__":
    main()
