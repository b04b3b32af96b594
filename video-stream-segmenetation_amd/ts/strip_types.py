"""Type-strip segment.ts into the Node module segment.js (CommonJS, Node 12).

This image has Node 12 and no TypeScript compiler, so the build ships a tiny,
deliberately narrow stripper for the subset segment.ts is written in:
  * `declare ...;` lines and `export interface X { ... }` blocks are dropped;
  * class field declarations without initialisers (`  name: Type;`) are dropped;
  * annotations are removed from function/method/arrow parameter lists, from
    return types (`): Type {`) and from `const|let name: Type =`;
  * `export class|function|const` lose `export`; a `module.exports = {...}`
    line lists them.
Anything outside the subset (casts, generic calls, object-literal types,
ternaries in if/while heads) is not supported; `node --check` on the output
and tests/test_ts.py guard it.

    python strip_types.py segment.ts > segment.js
"""
from __future__ import annotations

import re
import sys

KEYWORDS = {"if", "for", "while", "switch", "catch", "return", "function"}
TYPE = r"[A-Za-z_][\w.]*(?:<[^()]*?>)?(?:\[\])*(?:\s*\|\s*[A-Za-z_][\w.]*(?:<[^()]*?>)?(?:\[\])*)*"


def strip_params(params: str) -> str:
    out = []
    for p in params.split(","):
        m = re.match(r"^(\s*\.{0,3}\w+)\??\s*:\s*(" + TYPE + r")\s*(=.*)?$", p, re.S)
        if m:
            out.append(m.group(1) + (" " + m.group(3) if m.group(3) else ""))
        else:
            out.append(p)
    return ",".join(out)


def strip(src: str) -> str:
    lines = src.split("\n")
    out, exports, skip_block = [], [], False
    for line in lines:
        if skip_block:
            if line.startswith("}"):
                skip_block = False
            continue
        if re.match(r"^\s*declare\s", line):
            continue
        if re.match(r"^export interface \w+", line):
            skip_block = not line.rstrip().endswith("}")
            continue
        if re.match(r"^  \w+\??: " + TYPE + r";\s*$", line):
            continue  # class field declaration
        m = re.match(r"^export (class|function|const|let) (\w+)", line)
        if m:
            exports.append(m.group(2))
            line = line[len("export "):]
        out.append(line)
    text = "\n".join(out)

    # function / method / arrow parameter lists followed by a body or =>
    def fn_sub(m):
        name = m.group(1)
        if name in KEYWORDS - {"function"}:
            return m.group(0)
        return f"{name}({strip_params(m.group(2))})" + m.group(4)

    text = re.sub(r"(\bfunction\s*\w*|\b\w+)\s*\(([^()]*)\)(\s*:\s*" + TYPE + r")?(\s*(?:\{|=>))", fn_sub, text)
    text = re.sub(r"\b(const|let|var) (\w+): " + TYPE + r"( =)", r"\1 \2\3", text)
    if exports:
        text = text.rstrip("\n") + "\n\nmodule.exports = { " + ", ".join(exports) + " };\n"
    header = "// GENERATED from segment.ts by strip_types.py — edit segment.ts, not this file.\n'use strict';\n"
    return header + text


if __name__ == "__main__":
    sys.stdout.write(strip(open(sys.argv[1]).read()))
