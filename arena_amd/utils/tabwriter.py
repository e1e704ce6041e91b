"""Minimal Go text/tabwriter equivalent: tabwriter.NewWriter(w, 0, 0, 2, ' ', 0).

Cells are tab-terminated; a column's width is the widest cell of the consecutive block of lines
that have that column (Go semantics: a line with fewer cells ends the block for later columns).
Every cell terminated by a tab is padded to width + 2. The trailing cell (not tab-terminated) is
written as is. Output formats of list/get/top depend on this.
"""
from __future__ import annotations


class TabWriter:
    def __init__(self, out, padding: int = 2):
        self.out = out
        self.padding = padding
        self.buf = ""

    def write(self, s: str) -> None:
        self.buf += s

    def flush(self) -> None:
        lines = self.buf.split("\n")
        trailing_newline = self.buf.endswith("\n")
        if trailing_newline:
            lines = lines[:-1]
        rows = [ln.split("\t") for ln in lines]
        # cells[i][:-1] are tab-terminated; the last element is the trailing text
        widths = [[0] * (len(r) - 1) for r in rows]
        col = 0
        while True:
            active = False
            i = 0
            while i < len(rows):
                if len(rows[i]) - 1 > col:
                    active = True
                    j = i
                    w = 0
                    while j < len(rows) and len(rows[j]) - 1 > col:
                        w = max(w, len(rows[j][col]))
                        j += 1
                    for k in range(i, j):
                        widths[k][col] = w
                    i = j
                else:
                    i += 1
            if not active:
                break
            col += 1
        out = []
        for r, ws in zip(rows, widths):
            parts = [cell.ljust(w + self.padding) for cell, w in zip(r[:-1], ws)]
            out.append("".join(parts) + r[-1])
        text = "\n".join(out) + ("\n" if trailing_newline else "")
        self.out.write(text)
        self.buf = ""
