"""Resolve compile-time knobs of a C/HIP source at fixed values (a small unifdef).

    python tools/experiments/unifdef.py FILE -DNAME=VALUE ... [-o OUT]

Every ``#if/#elif/#else/#endif`` group whose conditions only involve the given
macros (``&&``, ``||``, ``!``, parentheses, integer literals, ``defined``) is
replaced by the branch that those values select; the ``#ifndef NAME / #define
NAME v / #endif`` default blocks of the given macros are dropped, and remaining
uses of them in ``#if`` lines or code keep their value.  Groups that involve
other macros are left as they are.  Used once to prune rwrt.hip of measured-
and-rejected variants (round 3); the variants stay in git history.
"""
import re
import sys


def parse_args(argv):
    defs, out, src = {}, None, None
    it = iter(argv)
    for a in it:
        if a.startswith("-D"):
            k, v = a[2:].split("=", 1)
            defs[k] = int(v)
        elif a == "-o":
            out = next(it)
        else:
            src = a
    return src, defs, out


TOK = re.compile(r"defined\s*\(\s*\w+\s*\)|defined\s+\w+|\w+|&&|\|\||!|\(|\)|==|!=|<=|>=|<|>|\+|-|\*")


def evaluate(expr, defs):
    """Python value of a preprocessor condition, or None if it names an unknown macro."""
    expr = re.sub(r"//.*", "", expr).strip()
    out = []
    for t in TOK.findall(expr):
        if t.startswith("defined"):
            name = re.sub(r"defined\s*\(?\s*(\w+)\s*\)?", r"\1", t)
            if name not in defs:
                return None
            out.append("True")
        elif t == "&&":
            out.append(" and ")
        elif t == "||":
            out.append(" or ")
        elif t == "!":
            out.append(" not ")
        elif re.fullmatch(r"\d+", t):
            out.append(t)
        elif re.fullmatch(r"\w+", t):
            if t not in defs:
                return None
            out.append(str(defs[t]))
        else:
            out.append(t)
    try:
        return bool(eval("".join(out)))
    except Exception:
        return None


def process(lines, defs):
    out = []
    # stack of frames: (mode, taken, emitting_parent)
    #   mode "keep": directive kept verbatim (unknown condition)
    #   mode "res":  resolved; `active` = this branch is emitted, `done` = a branch was taken
    stack = []

    def emitting():
        return all(f["active"] for f in stack)

    i = 0
    while i < len(lines):
        ln = lines[i]
        m = re.match(r"\s*#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)", ln)
        if not m:
            if emitting():
                out.append(ln)
            i += 1
            continue
        kw, rest = m.group(1), m.group(2)
        if kw == "ifndef" and rest.split()[0] in defs:
            # the knob's default block: #ifndef X / #define X v / #endif -> drop
            name = rest.split()[0]
            j = i + 1
            while not re.match(r"\s*#\s*endif", lines[j]):
                j += 1
            i = j + 1
            continue
        if kw in ("if", "ifdef", "ifndef"):
            if kw == "if":
                val = evaluate(rest, defs)
            elif kw == "ifdef":
                val = True if rest.split()[0] in defs else None
            else:
                val = None
            if val is None:
                stack.append({"mode": "keep", "active": True, "done": False})
                if emitting():
                    out.append(ln)
            else:
                stack.append({"mode": "res", "active": val, "done": val})
            i += 1
            continue
        f = stack[-1]
        if kw == "elif":
            if f["mode"] == "keep":
                if all(g["active"] for g in stack[:-1]):
                    out.append(ln)
            else:
                val = evaluate(rest, defs)
                if val is None:
                    raise SystemExit(f"line {i + 1}: #elif with an unknown macro after a resolved #if")
                f["active"] = (not f["done"]) and val
                f["done"] = f["done"] or val
        elif kw == "else":
            if f["mode"] == "keep":
                if all(g["active"] for g in stack[:-1]):
                    out.append(ln)
            else:
                f["active"] = not f["done"]
                f["done"] = True
        elif kw == "endif":
            stack.pop()
            if f["mode"] == "keep" and emitting():
                out.append(ln)
        i += 1
    assert not stack, "unbalanced conditionals"
    return out


def main():
    src, defs, out = parse_args(sys.argv[1:])
    lines = open(src).read().split("\n")
    res = process(lines, defs)
    text = "\n".join(res)
    # remaining plain uses of the knobs in code take their value
    # (code only: comments that name a knob are left for a human to rewrite)
    lines = []
    for ln in text.split("\n"):
        code, sep, com = ln.partition("//")
        for k, v in defs.items():
            code = re.sub(r"\b%s\b" % k, str(v), code)
        lines.append(code + sep + com)
    text = "\n".join(lines)
    text = re.sub(r"\n{3,}", "\n\n", text)
    open(out or src, "w").write(text)


if __name__ == "__main__":
    main()
