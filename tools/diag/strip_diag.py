"""Round 6: move the diagnostic hooks (OLPE_DIAG_* / OLPE_EXP_* conditionals and the
DT_MARK section timers) out of the product kernel sources into a patch.

    python tools/diag/strip_diag.py            # strip in place, write diag_hooks.patch

Every conditional whose expression names only OLPE_DIAG_* / OLPE_EXP_* macros is
resolved with those macros undefined (the product build); DT_MARK(i); statements and
the no-op DT_MARK definition go too.  The patch (tools/diag/diag_hooks.patch) turns the
stripped sources back into the hooked ones: tools/diag_build.sh applies it to a copy of
the sources, never to the tree.  The product code object is unchanged by construction
(kernel_digest e9c2fc13a6f6bbf5 before and after, checked when the hooks were moved in
round 6; tests/test_abi.py::test_product_sources_carry_no_diagnostic_hooks keeps the
sources free of them and the patch applicable)."""
from __future__ import annotations

import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FILES = ["olpefit_amd/csrc/olpe.hip", "olpefit_amd/csrc/olpe_device.h"]
DIAG = re.compile(r"\bOLPE_(DIAG|EXP)_\w+")
COND = re.compile(r"^\s*#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)$")


def _eval(kind: str, expr: str) -> bool | None:
    """Truth of a diag-only condition with every diag macro undefined; None if the
    condition names anything else."""
    expr = expr.split("//")[0].strip()
    if kind in ("ifdef", "ifndef"):
        if not DIAG.fullmatch(expr):
            return None
        return kind == "ifndef"
    rest = DIAG.sub("", re.sub(r"defined\s*\(\s*OLPE_(DIAG|EXP)_\w+\s*\)", "0", expr))
    if re.search(r"[A-Za-z_]", rest.replace("0", "")):
        return None
    py = re.sub(r"defined\s*\(\s*OLPE_(DIAG|EXP)_\w+\s*\)", "False", expr)
    py = py.replace("&&", " and ").replace("||", " or ").replace("!", " not ")
    return bool(eval(py, {}, {}))        # noqa: S307 -- our own source's #if lines


def strip(text: str) -> str:
    out = []
    stack = []          # per open conditional: None (not diag) or [taking, taken_any]
    for line in text.splitlines(keepends=True):
        m = COND.match(line)
        live = all(f is None or f[0] for f in stack)
        if m:
            kind, expr = m.group(1), m.group(2)
            if kind in ("if", "ifdef", "ifndef"):
                v = _eval(kind, expr)
                stack.append(None if v is None else [v, v])
                if v is None and live:
                    out.append(line)
                continue
            top = stack[-1]
            if kind == "elif":
                if top is None:
                    if live:
                        out.append(line)
                    continue
                v = _eval("if", expr)
                assert v is not None, line
                top[0] = (not top[1]) and v
                top[1] = top[1] or v
                continue
            if kind == "else":
                if top is None:
                    if all(f is None or f[0] for f in stack[:-1]):
                        out.append(line)
                    continue
                top[0] = not top[1]
                top[1] = True
                continue
            stack.pop()                               # endif
            if top is None and all(f is None or f[0] for f in stack):
                out.append(line)
            continue
        if live:
            out.append(line)
    assert not stack
    s = "".join(out)
    # the section timers: their no-op definition and every DT_MARK(i); statement
    s = re.sub(r"#define DT_MARK\(i\) \\\n  do \{             \\\n  \} while \(0\)\n", "", s)
    s = re.sub(r"^[ \t]*DT_MARK\(\d+\);[ \t]*\n", "", s, flags=re.M)
    assert "DT_MARK" not in s, "DT_MARK left"
    return s


def main():
    patch = []
    for rel in FILES:
        path = os.path.join(REPO, rel)
        with open(path) as f:
            orig = f.read()
        new = strip(orig)
        if new == orig:
            continue
        tmp = path + ".stripped"
        with open(tmp, "w") as f:
            f.write(new)
        d = subprocess.run(["diff", "-u", "--label", f"a/{rel}", "--label", f"b/{rel}", tmp,
                            path], capture_output=True, text=True)
        patch.append(d.stdout)
        os.replace(tmp, path)
    if patch:
        with open(os.path.join(REPO, "tools", "diag", "diag_hooks.patch"), "w") as f:
            f.write("".join(patch))
    print("stripped" if patch else "nothing to strip", file=sys.stderr)


if __name__ == "__main__":
    main()
