#!/usr/bin/env python3
"""Per-op cost of the interpreter kernels (diagnostic, not the driver's bench).

Each probe program is REPS copies of one instruction followed by `exit`, run over 1 Mi 64-byte
frames; all lanes of a wave execute every micro-op, so (t(probe) - t(exit only)) / REPS is the
chip-wide cost of one wave-iteration of that op kind, for 16384 waves. Prints one JSON line per
kernel (fast path and general interpreter) with microseconds per launch and nanoseconds per
iteration step (per 1 Mi packets).

  python tools/opcost.py [--reps 60] [--launches 100]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))

PROBES = {
    "exit": "",
    "mov64_imm": "mov r3, 7",
    "add64_imm": "add r3, 7",
    "add64_reg": "add r3, r4",
    "and32_imm": "and32 r3, 0xff",
    "lsh64_imm": "lsh r3, 2",
    "be16": "be16 r3",
    "ldxb": "ldxb r3, [r1+14]",
    "ldxh": "ldxh r3, [r1+12]",
    "ldxw": "ldxw r3, [r1+26]",
    "ldxdw": "ldxdw r3, [r1+8]",
    "ja": "ja +0",
    "jeq_imm": "jeq r3, 99, +0",
    "jne_imm": "jne r3, 99, +0",
    "jgt_reg": "jgt r3, r4, +0",
    "jlt_imm": "jlt r3, 20, +0",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=60)
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--only", default="", help="comma list of probe names")
    args = ap.parse_args()

    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    dev = torch.device("cuda", 0)
    n = args.packets
    frames = torch.from_numpy(W.frames_fixed(n, 64, 3)).to(dev)
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    names = [p for p in args.only.split(",") if p] or list(PROBES)
    if "exit" not in names:
        names = ["exit"] + names

    def timed(prog, generic):
        b = prog.make_batch(frames, n=n, stride=64, generic=generic)
        out = _lib.BatchOut()
        out.verdict = verdict.data_ptr()
        out.counters = counters.data_ptr()
        for _ in range(5):
            prog.launch(b, out, stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(args.launches):
            prog.launch(b, out, stream)
        ev[1].record(stream)
        torch.cuda.synchronize(dev)
        return ev[0].elapsed_time(ev[1]) * 1e3 / args.launches  # us per launch

    for generic in (False, True):
        res = {}
        for name in names:
            body = (PROBES[name] + "\n") * args.reps if PROBES[name] else ""
            prog = Program(assemble(body + "exit"))
            res[name] = timed(prog, generic)
            prog.close()
        base = res["exit"]
        per = {k: round((v - base) / args.reps * 1e3, 1) for k, v in res.items() if k != "exit"}
        print(json.dumps({"kernel": "general" if generic else "fast",
                          "us_exit_only": round(base, 2),
                          "ns_per_step_per_1Mi": per,
                          "us_per_launch": {k: round(v, 2) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
