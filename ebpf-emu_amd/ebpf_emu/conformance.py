"""bpf_conformance `.data` runner.

The reference is validated only by the external Alan-Jowett/bpf_conformance suite (notes.md:4-19,
.gitmodules:1-3), whose vectors are absent from this environment. This module reads that suite's
`.data` format -- `-- asm` (ubpf syntax) or `-- raw` (hex words), `-- mem` (hex bytes), `-- result`
(expected r0) or `-- error` (expected failure) -- and runs every vector through the GPU path with
the reference harness layout (main.rs:14-31), so the suite can pin parity wherever it exists:

    python -m ebpf_emu.conformance path/to/bpf_conformance/tests [--exclude-groups atomic64]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
from dataclasses import dataclass

from .asm import assemble


@dataclass
class Vector:
    name: str
    program: bytes
    memory: bytes
    result: int | None
    expect_error: bool


def parse_data(text: str, name: str = "") -> Vector:
    sections: dict[str, list[str]] = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^--\s*(\w+)", line)
        if m:
            cur = m.group(1).lower()
            sections.setdefault(cur, [])
            continue
        if cur is not None:
            sections[cur].append(line)
    if "raw" in sections:
        hexs = "".join(sections["raw"]).replace(" ", "").replace("\t", "")
        words = [hexs[i:i + 16] for i in range(0, len(hexs), 16)]
        program = b"".join(bytes.fromhex(w) for w in words)
    else:
        program = assemble("\n".join(sections.get("asm", [])))
    mem_hex = "".join(l.split("#")[0] for l in sections.get("mem", [])).replace(" ", "").strip()
    memory = bytes.fromhex(mem_hex) if mem_hex else b""
    result = None
    res_txt = " ".join(l.split("#")[0].strip() for l in sections.get("result", [])).strip()
    if res_txt:
        result = int(res_txt, 0) & ((1 << 64) - 1)
    return Vector(name, program, memory, result, "error" in sections)


def run_vector(v: Vector, device: int = 0):
    """-> (passed, status, r0) using the emem harness layout (memory image = the packet)."""
    import torch

    from ._lib import DEFAULT_MEM
    from .ins import DecodeError
    from .program import Program

    try:
        prog = Program(v.program)
    except DecodeError:
        return v.expect_error, -1, None
    if len(v.memory) > DEFAULT_MEM:
        return v.expect_error, 7, None
    dev = torch.device("cuda", device)
    frames = torch.zeros(max(8, len(v.memory)), dtype=torch.uint8, device=dev)
    if v.memory:
        frames[:len(v.memory)] = torch.tensor(list(v.memory), dtype=torch.uint8)
    lens = torch.tensor([len(v.memory)], dtype=torch.int16, device=dev)
    res = prog.run(frames, n=1, stride=frames.numel(), lens=lens, verdict=False, r0=True, status=True)
    torch.cuda.synchronize(dev)
    st = int(res.status[0].item())
    r0 = int(res.r0[0].item()) & ((1 << 64) - 1)
    prog.close()
    if v.expect_error:
        return st != 0, st, r0
    return st == 0 and (v.result is None or r0 == v.result), st, r0


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--exclude-groups", default="", help="comma list of name prefixes to skip")
    args = ap.parse_args(argv)
    files = []
    for p in args.paths:
        files += sorted(glob.glob(os.path.join(p, "*.data"))) if os.path.isdir(p) else [p]
    skip = [g for g in args.exclude_groups.split(",") if g]
    passed = failed = 0
    fails = []
    for f in files:
        name = os.path.basename(f)
        if any(name.startswith(g) for g in skip):
            continue
        with open(f) as fh:
            v = parse_data(fh.read(), name)
        ok, st, r0 = run_vector(v)
        passed += ok
        failed += not ok
        if not ok:
            fails.append({"test": name, "status": st, "r0": None if r0 is None else f"{r0:x}"})
    print(json.dumps({"passed": passed, "total": passed + failed, "failures": fails}))
    return 0 if failed == 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
