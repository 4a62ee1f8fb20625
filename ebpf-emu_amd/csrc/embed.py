#!/usr/bin/env python3
"""Embeds a text file (the JIT template kernels' assembly, build/tile_jit.s) as a C string.

  python3 embed.py <input> <output.h> <symbol>
"""
import sys


def main():
    src, dst, sym = sys.argv[1:4]
    text = open(src).read()
    lines = ['"' + ln.replace("\\", "\\\\").replace('"', '\\"').replace("\t", "\\t") + '\\n"'
             for ln in text.splitlines()]
    with open(dst, "w") as f:
        f.write(f"// GENERATED from {src} by embed.py -- do not edit.\n#pragma once\n")
        f.write(f"static const char {sym}[] =\n" + "\n".join(lines) + ";\n")


if __name__ == "__main__":
    main()
