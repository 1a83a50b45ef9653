"""Resolve rejected code-shape flags in a source file to their kept values
(a small `unifdef`: none is installed in this image).

    python scripts/prune_flags.py FILE NAME=VALUE ...

Conditionals whose expression becomes constant are resolved (their dead
branches dropped); the others keep their directive with the resolved names
replaced by their values.  Non-directive lines get `LZGPU_NAME` replaced by the
value too (for `if constexpr (LZGPU_X && ...)`)."""
import re
import sys


def parse_expr(e, vals):
    """Evaluate a directive expression with the resolved flags; None if it
    depends on anything else."""
    e = e.split("//")[0].strip()
    unknown = False

    def sub_defined(m):
        nonlocal unknown
        name = m.group(1)
        if name in vals:
            return "1"
        unknown = True
        return "0"

    e2 = re.sub(r"defined\s*\(\s*(\w+)\s*\)", sub_defined, e)
    e2 = re.sub(r"defined\s+(\w+)", sub_defined, e2)

    def sub_name(m):
        nonlocal unknown
        name = m.group(0)
        if name in vals:
            return str(vals[name])
        if re.fullmatch(r"0x[0-9a-fA-F]+u?|\d+u?", name):
            return name.rstrip("u")
        unknown = True
        return "0"

    e3 = re.sub(r"\b[A-Za-z_]\w*\b|0x[0-9a-fA-F]+u?|\b\d+u?\b", sub_name, e2)
    if unknown:
        return None
    py = e3.replace("&&", " and ").replace("||", " or ").replace("!", " not ")
    py = py.replace(" not =", "!=")
    return bool(eval(py))


def substitute(line, vals):
    def sub(m):
        return str(vals[m.group(0)]) if m.group(0) in vals else m.group(0)
    return re.sub(r"\bLZGPU_\w+\b", sub, line)


def prune(text, vals):
    out = []
    # stack entries: [state, any_taken, keep_directive]; state: True emit, False drop
    stack = []

    def emitting():
        return all(s[0] for s in stack)

    for line in text.split("\n"):
        m = re.match(r"\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", line)
        if not m:
            if emitting():
                out.append(substitute(line, vals))
            continue
        kw, rest = m.group(1), m.group(2).strip()
        if kw in ("if", "ifdef", "ifndef"):
            if kw == "ifdef":
                v = True if rest.split()[0] in vals else None
            elif kw == "ifndef":
                v = False if rest.split()[0] in vals else None
            else:
                v = parse_expr(rest, vals)
            if v is None:
                stack.append([True, False, True])
                if emitting():
                    out.append(substitute(line, vals))
            else:
                stack.append([v, v, False])
        elif kw == "elif":
            top = stack[-1]
            if top[2]:
                # the chain is kept: an elif of a kept chain stays as written
                v = parse_expr(rest, vals)
                if v is False:
                    top[0] = False
                else:
                    top[0] = True
                    stack.pop()
                    if emitting():
                        out.append(substitute(line, vals))
                    stack.append(top)
                continue
            if top[1]:
                top[0] = False
            else:
                v = parse_expr(rest, vals)
                if v is None:
                    # first undecided elif of a resolved chain becomes an #if
                    top[0], top[1], top[2] = True, True, True
                    stack.pop()
                    if emitting():
                        out.append(re.sub(r"#\s*elif", "#if", substitute(line, vals), count=1))
                    stack.append(top)
                else:
                    top[0], top[1] = v, v
        elif kw == "else":
            top = stack[-1]
            if top[2]:
                stack.pop()
                if emitting():
                    out.append(line)
                top[0] = True
                stack.append(top)
            else:
                top[0] = not top[1]
                top[1] = True
        else:  # endif
            top = stack.pop()
            if top[2] and emitting():
                out.append(line)
    assert not stack, "unbalanced conditionals"
    return "\n".join(out)


def main():
    path = sys.argv[1]
    vals = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=")
        vals[k] = int(v, 0)
    src = open(path).read()
    open(path, "w").write(prune(src, vals))


if __name__ == "__main__":
    main()
