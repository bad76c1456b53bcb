#!/usr/bin/env python3
"""Minimal unifdef for the kernel sources: resolve the preprocessor conditionals that test ONLY the given macros
(fixed to their product values, or undefined), keep every other conditional as written, and substitute the fixed
macros' values where code uses them outside directives. Used once (round 6) to move rejected experiment branches out
of the shipped kernels; the removed text is kept as a reverse patch under diag/ (git diff of the change).

    python3 diag/strip_knobs.py FILE -D NAME=VALUE ... -U NAME ...
"""
import re
import sys

IDENT = re.compile(r"\b[A-Za-z_][A-Za-z0-9_]*\b")


def evaluate(expr, defs, undefs):
    """True / False when expr only involves known macros, else None."""
    e = re.sub(r"//.*", "", expr).strip()

    def dfn(m):
        n = m.group(1)
        if n in defs:
            return "1"
        if n in undefs:
            return "0"
        raise KeyError(n)
    try:
        e = re.sub(r"defined\s*\(?\s*([A-Za-z_][A-Za-z0-9_]*)\s*\)?", dfn, e)
    except KeyError:
        return None
    for n in set(IDENT.findall(e)):
        if n in defs:
            e = re.sub(r"\b%s\b" % n, str(defs[n]), e)
        elif n in undefs:
            e = re.sub(r"\b%s\b" % n, "0", e)
        else:
            return None
    e = e.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace("not =", "!=")
    return bool(eval(e))  # noqa: S307 (expressions of integer literals only)


def strip(lines, defs, undefs):
    out = []
    # stack entries: [mode, taken] with mode "keep" (unknown: directive lines kept) or "fixed" (resolved),
    # emit = whether lines in the current branch are emitted
    stack = []

    def emitting():
        return all(s["emit"] for s in stack)
    for ln in lines:
        m = re.match(r"\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", ln)
        if not m:
            if emitting():
                if not re.match(r"\s*#\s*undef\b", ln):
                    for n, v in defs.items():
                        ln = re.sub(r"\b%s\b" % n, str(v), ln)
                out.append(ln)
            continue
        d, rest = m.group(1), m.group(2)
        if d in ("if", "ifdef", "ifndef"):
            if d == "ifdef":
                val = evaluate("defined(%s)" % rest.strip().split()[0], defs, undefs)
            elif d == "ifndef":
                v = evaluate("defined(%s)" % rest.strip().split()[0], defs, undefs)
                val = None if v is None else not v
            else:
                val = evaluate(rest, defs, undefs)
            if val is None:
                stack.append({"mode": "keep", "emit": True, "taken": False})
                if emitting():
                    out.append(ln)
            else:
                stack.append({"mode": "fixed", "emit": val, "taken": val})
        elif d == "elif":
            s = stack[-1]
            if s["mode"] == "keep":
                if all(x["emit"] for x in stack[:-1]):
                    out.append(ln)
                continue
            val = evaluate(rest, defs, undefs)
            if val is None:
                raise SystemExit("unresolvable #elif after a resolved #if: " + ln)
            s["emit"] = (not s["taken"]) and val
            s["taken"] = s["taken"] or val
        elif d == "else":
            s = stack[-1]
            if s["mode"] == "keep":
                if all(x["emit"] for x in stack[:-1]):
                    out.append(ln)
                continue
            s["emit"] = not s["taken"]
            s["taken"] = True
        else:
            s = stack.pop()
            if s["mode"] == "keep" and emitting():
                out.append(ln)
    assert not stack, "unbalanced conditionals"
    return out


def main():
    path = sys.argv[1]
    defs, undefs = {}, set()
    a = sys.argv[2:]
    i = 0
    while i < len(a):
        if a[i] == "-D":
            n, _, v = a[i + 1].partition("=")
            defs[n] = v or "1"
            i += 2
        elif a[i] == "-U":
            undefs.add(a[i + 1])
            i += 2
        else:
            raise SystemExit("bad argument " + a[i])
    with open(path) as f:
        lines = f.read().split("\n")
    with open(path, "w") as f:
        f.write("\n".join(strip(lines, defs, undefs)))


if __name__ == "__main__":
    main()
