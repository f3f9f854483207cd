"""A structural check of Go source for a container without a Go toolchain (no `go`, no `gofmt`).

It tokenizes comments, strings (interpreted and raw) and runes, then checks what a hand-edited diff hunk breaks
(top-level functions landed inside `type Implementation interface {`):

* (), [] and {} balance and nest, and every file ends at depth 0;
* `package` comes first, and `func` / `type` / `var` / `const` / `import` in column 0 only occur at depth 0;
* gofmt indentation: a line that starts at brace depth d outside parentheses starts with d tabs (closing lines and
  `case` / `default` labels d-1, goto labels any), and no line mixes leading spaces into its indent.

It is calibrated on the reference's own gofmt'd sources (tests/test_integration_go.py runs it over every Go file in
/root/reference when present), so a failure means the edited file would not survive `gofmt -e`.
"""
import re

_OPEN = {"(": ")", "[": "]", "{": "}"}
_CLOSE = {v: k for k, v in _OPEN.items()}


def _strip(src):
    """src with comments, strings and runes blanked (newlines kept), so brackets and keywords can be scanned."""
    out = []
    i, n = 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            out.append(" " * (j - i))
            i = j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            if j < 0:
                raise SyntaxError("unterminated block comment")
            out.append("".join(ch if ch == "\n" else " " for ch in src[i:j + 2]))
            i = j + 2
        elif c == "`":
            j = src.find("`", i + 1)
            if j < 0:
                raise SyntaxError("unterminated raw string")
            out.append('"' + "".join(ch if ch == "\n" else " " for ch in src[i + 1:j]) + '"')
            i = j + 1
        elif c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                if src[j] == "\n":
                    raise SyntaxError("newline in string or rune at offset %d" % i)
                j += 2 if src[j] == "\\" else 1
            if j >= n:
                raise SyntaxError("unterminated string or rune")
            out.append(c + " " * (j - i - 1) + c)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def check(src, name="<go>"):
    """Raise SyntaxError naming the line of the first structural fault of `src`."""
    code = _strip(src)
    lines = code.split("\n")
    raw = src.split("\n")
    # lines that continue a multi-line raw string are data, not code
    inraw, q = set(), False
    for no, rl in enumerate(raw, 1):
        if q:
            inraw.add(no)
        if rl.count("`") % 2 and not rl.lstrip().startswith("//"):
            q = not q
    first = next((ln for ln in lines if ln.strip()), "")
    if not first.startswith("package "):
        raise SyntaxError("%s: the first statement is not `package`" % name)
    stack = []  # (char, line, indent of the statement that opened it)
    prev = ""
    cont = None  # the statement indent when this line continues the previous one
    for no, (ln, rl) in enumerate(zip(lines, raw), 1):
        s = ln.strip()
        lead = rl[:len(rl) - len(rl.lstrip(" \t"))]
        cont = None
        if s and no not in inraw:
            if re.match(r"(func|type|var|const|import)\b", ln) and stack:
                raise SyntaxError("%s:%d: top-level `%s` at depth %d (opened at line %d)"
                                  % (name, no, ln.split()[0], len(stack), stack[-1][1]))
            if " " in lead and (not stack or stack[-1][0] == "{"):
                raise SyntaxError("%s:%d: spaces in the indentation" % (name, no))
            if stack and stack[-1][0] == "{":
                base = stack[-1][2]
                want = base if s[0] == "}" else base + 1
                tabs = len(lead)
                ok = tabs == want
                ok = ok or (re.match(r"(case\b|default\s*:)", s) and tabs == want - 1)
                ok = ok or re.match(r"[A-Za-z_]\w*:\s*$", s)  # goto label
                if not ok and tabs == want + 1 and re.search(r"(\|\||&&|[-+*/|&.,=:])\s*$", prev):
                    ok, cont = True, want  # a continuation line: braces it opens close at the statement's indent
                if not ok:
                    raise SyntaxError("%s:%d: indent %d tabs, want %d" % (name, no, tabs, want))
            elif not stack and s[0] not in ")]}" and lead:
                raise SyntaxError("%s:%d: indented line at top level" % (name, no))
        start = stack[-1][2] if stack and stack[-1][0] in "([" else None  # the line continues a call's arguments
        for ch in ln:
            if ch in _OPEN:
                if cont is not None:
                    stmt = cont
                elif ch == "{" and start is not None and (not stack or stack[-1][0] == "{"):
                    stmt = start  # `...); err != nil {` closes the arguments, then opens the statement's block
                else:
                    stmt = len(lead)
                stack.append((ch, no, stmt))
            elif ch in _CLOSE:
                if not stack or stack[-1][0] != _CLOSE[ch]:
                    raise SyntaxError("%s:%d: unbalanced `%s`" % (name, no, ch))
                stack.pop()
        if s and no not in inraw:
            prev = s
    if stack:
        raise SyntaxError("%s: `%s` opened at line %d is never closed" % (name, stack[-1][0], stack[-1][1]))
