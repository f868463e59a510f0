"""Minimal unifdef: resolve #if / #elif / #else / #endif blocks whose conditions use only the given
macros (and integer literals), leave every other conditional untouched.  Used to fold the settled
compile-time A/B switches into fixed code.  Usage: unifdef.py FILE NAME=VALUE ..."""
import re
import sys


def evaluate(cond, defs):
    c = cond.strip()
    c = re.sub(r"//.*", "", c)
    toks = re.findall(r"[A-Za-z_]\w*", c)
    for t in toks:
        if t not in defs:
            return None
    expr = c
    for t in sorted(set(toks), key=len, reverse=True):
        expr = re.sub(r"\b%s\b" % t, str(defs[t]), expr)
    expr = expr.replace("&&", " and ").replace("||", " or ")
    expr = re.sub(r"!(?!=)", " not ", expr)
    try:
        return bool(eval(expr, {}, {}))
    except Exception:
        return None


def process(lines, defs):
    out = []
    # stack entries: (mode, emitting_before, taken) ; mode 'keep' = unresolved (copy directives)
    stack = []
    emit = True
    for ln in lines:
        s = ln.strip()
        m = re.match(r"#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)", s)
        if not m:
            if emit:
                out.append(ln)
            continue
        d, rest = m.group(1), m.group(2)
        if d in ("ifndef", "ifdef"):
            name = rest.strip().split()[0]
            if name in defs and d == "ifndef":
                # "#ifndef X / #define X v / #endif" guard: drop it entirely
                stack.append(("res", emit, True, False))
                emit = False
                continue
            stack.append(("keep", emit, None, None))
            if emit:
                out.append(ln)
            continue
        if d == "if":
            v = evaluate(rest, defs)
            if v is None:
                stack.append(("keep", emit, None, None))
                if emit:
                    out.append(ln)
            else:
                stack.append(("res", emit, v, True))
                emit = emit and v
            continue
        top = stack[-1]
        if d == "elif":
            if top[0] == "keep":
                if top[1]:
                    out.append(ln)
                continue
            v = evaluate(rest, defs)
            assert v is not None, ln
            taken = top[2]
            stack[-1] = ("res", top[1], taken or v, True)
            emit = top[1] and (not taken) and v
            continue
        if d == "else":
            if top[0] == "keep":
                if top[1]:
                    out.append(ln)
                continue
            taken = top[2]
            stack[-1] = ("res", top[1], True, True)
            emit = top[1] and not taken and top[3] is not False
            continue
        if d == "endif":
            stack.pop()
            if top[0] == "keep":
                if top[1]:
                    out.append(ln)
            emit = top[1]
            continue
    assert not stack
    return out


if __name__ == "__main__":
    path = sys.argv[1]
    defs = {}
    for a in sys.argv[2:]:
        k, v = a.split("=")
        defs[k] = int(v)
    lines = open(path).read().split("\n")
    open(path, "w").write("\n".join(process(lines, defs)))
