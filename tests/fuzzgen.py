"""Seeded random program / packet generator for differential tests (test infrastructure).

Programs mix every instruction class the reference decodes: ALU/ALU64 (all 14 ops, imm and
register sources, END widths incl. invalid ones), JMP/JMP32 (forward and occasional backward
offsets, so some programs loop into the step budget), LDX/ST/STX/ATOMIC around the packet, the
stack and the image end, wide lddw of edge values, CALL/EXIT, register 11 and a few opcodes that
fault at run time. `valid_only=False` also produces load-time rejects.
"""
from __future__ import annotations

import random

from ebpf_emu.asm import encode

EDGE = [0, 1, 2, 7, 0x7F, 0x80, 0xFF, 0x100, 0x7FFF, 0x8000, 0xFFFF, 0x7FFFFFFF, 0x80000000,
        0xFFFFFFFF, 0x100000000, 0x7FFFFFFFFFFFFFFF, 0x8000000000000000, 0xFFFFFFFFFFFFFFFF,
        0xFFFFFFFF00000000, 0x0000000100000001, 512, 504, 1016, 1020, 1023, 1024]
IMM_EDGE = [0, 1, -1, 2, 7, 8, 16, 31, 32, 33, 63, 64, 65, -4, 0x7FFFFFFF, -0x80000000, 0x11, 53,
            1024, 1020, 1023, 100]
ATOMIC_IMMS = [0x00, 0x01, 0x40, 0x41, 0x50, 0x51, 0xA0, 0xA1, 0xE1, 0xF1, 0xE0, 0xF0, 0x10, 0x100]


def _reg(rng, allow11=0.01):
    if rng.random() < allow11:
        return 11
    return rng.randrange(11)


def _imm(rng):
    if rng.random() < 0.6:
        return rng.choice(IMM_EDGE)
    return rng.randrange(-(1 << 31), 1 << 31)


def _mem_ref(rng):
    """(base register, offset) aimed at the packet, the stack or the image edges."""
    k = rng.random()
    if k < 0.45:
        return 1, rng.randrange(-2, 72)
    if k < 0.8:
        return 10, -rng.randrange(1, 64)
    if k < 0.9:
        return 1, rng.choice([1016, 1017, 1020, 1021, 1023, 1024, 2000, -8])
    return rng.randrange(11), rng.randrange(-64, 64)


def gen_program(rng: random.Random, n: int | None = None, valid_only: bool = True,
                allow_loops: bool = True, tier0: bool = False) -> bytes:
    """tier0=True: no ST/STX/ATOMIC/CALL (the read-only memory tier); with allow_loops=False
    every jump goes forward, i.e. the program qualifies for the forward-jump fast path."""
    n = n or rng.randrange(3, 40)
    words: list[bytes] = []
    # seed registers with edge values so arithmetic corners are reached
    for r in rng.sample([0, 3, 4, 5, 6, 7, 8, 9], rng.randrange(0, 4)):
        v = rng.choice(EDGE)
        words.append(encode(0x18, r, 0, 0, v & 0xFFFFFFFF) + encode(0, 0, 0, 0, v >> 32))
    while len(words) < n:
        k = rng.random()
        dst, src = _reg(rng), _reg(rng)
        if k < 0.40:  # ALU / ALU64
            cls = rng.choice([0x04, 0x07])
            op = rng.randrange(14)
            srcbit = rng.choice([0, 0x08])
            if op == 13:
                imm = rng.choice([16, 32, 64, 16, 32, 64, 8, 0])
                words.append(encode((op << 4) | srcbit | cls, dst, 0, 0, imm))
            else:
                words.append(encode((op << 4) | srcbit | cls, dst, src, 0, _imm(rng)))
        elif k < 0.60:  # JMP / JMP32
            cls = rng.choice([0x05, 0x06])
            op = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 10, 11, 12, 13])
            remaining = max(1, n - len(words))
            off = rng.randrange(0, remaining + 2)
            if allow_loops and rng.random() < 0.05:
                off = -rng.randrange(1, 4)
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, off, _imm(rng)))
        elif k < 0.72:  # LDX
            base, off = _mem_ref(rng)
            size = rng.choice([0x00, 0x08, 0x10, 0x18])
            words.append(encode(0x61 | size, dst, base, off))
        elif k < 0.80 and tier0:
            continue
        elif k < 0.80:  # ST / STX
            base, off = _mem_ref(rng)
            size = rng.choice([0x00, 0x08, 0x10, 0x18])
            if rng.random() < 0.5:
                words.append(encode(0x62 | size, base, 0, off, _imm(rng)))
            else:
                words.append(encode(0x63 | size, base, src, off))
        elif k < 0.86 and tier0:
            continue
        elif k < 0.86:  # ATOMIC
            base, off = (10, -8 * rng.randrange(1, 6)) if rng.random() < 0.8 else _mem_ref(rng)
            size = rng.choice([0x00, 0x18, 0x18, 0x08])
            cls = 0x03 if rng.random() < 0.9 else 0x02
            words.append(encode(0xC0 | size | cls, base, src, off, rng.choice(ATOMIC_IMMS)))
        elif k < 0.90:  # lddw
            v = rng.choice(EDGE) if rng.random() < 0.7 else rng.getrandbits(64)
            words.append(encode(0x18, dst, 0, 0, v & 0xFFFFFFFF) + encode(0, 0, 0, 0, v >> 32))
        elif k < 0.93:  # CALL / EXIT
            if rng.random() < 0.5 and not tier0:
                words.append(encode(0x85, 0, 0, rng.randrange(0, 4)))
            else:
                words.append(encode(0x95))
        elif k < 0.96:  # run-time faults
            words.append(rng.choice([encode(0x20, 0, 0, 0, 0), encode(0x60, 0, 1, 0),
                                     encode(0xD9, 0, 1, 0), encode(0x8D, 0, 1, 0),
                                     encode(0x1A, 0, 0, 0, 0) + bytes(8)]))
        else:  # mov
            words.append(encode(0xB7 | rng.choice([0, 0x08]), dst, src, 0, _imm(rng)))
        if not valid_only and rng.random() < 0.02:
            words.append(rng.choice([encode(0xE7), encode(0x81, 0, 1), encode(0xB7, 12, 0),
                                     encode(0xE1, 0, 1)]))
    if rng.random() < 0.9:
        words.append(encode(0x95))
    return b"".join(words)


def gen_packet(rng: random.Random, max_len: int = 80) -> bytes:
    n = rng.choice([0, 1, 2, 5, 14, 34, 60, 63, 64, 65, rng.randrange(0, max_len + 1)])
    return bytes(rng.getrandbits(8) for _ in range(n))


def gen_stack_program(rng: random.Random, n: int | None = None, k: int = 32,
                      pw_atomics: bool = False) -> bytes:
    """Forward-only programs whose stores all hit the stack window [r10 - k, r10) (memory tier
    0.5): ST/STX of every width at aligned and misaligned r10 offsets, directly and through a copy
    of r10 (`mov r9, r10; add r9, -c`), loads of the window at r10 offsets, loads of the packet,
    and register-address loads aimed just below and into the window through r1 (the store-
    forwarding overlay, r10 = 512 in the main.rs layout) -- mixed with ALU ops and forward jumps.
    pw_atomics: also stack atomics (every operation, 32/64-bit, with and without fetch, at aligned
    r10 offsets) and ST/STX into the packet's first 64 bytes, without register-address loads."""
    n = n or rng.randrange(6, 40)
    words: list[bytes] = []
    if rng.random() < 0.5:  # a second pointer into the stack
        c = rng.randrange(0, 9)
        words.append(encode(0xBF, 9, 10, 0, 0))         # mov r9, r10
        words.append(encode(0x07, 9, 0, 0, -c))         # add r9, -c
    else:
        c = None
    sizes = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}
    while len(words) < n:
        q = rng.random()
        dst = rng.randrange(9)
        src = rng.randrange(10)
        size = rng.choice(list(sizes))
        w = sizes[size]
        if pw_atomics and q < 0.12:  # an atomic on the window, or a packet-window store
            if rng.random() < 0.5:
                d = -4 * rng.randrange(2, k // 4 + 1)
                base, off = (10, d) if c is None or rng.random() < 0.5 else (9, d + c)
                aop = rng.choice([0x00, 0x40, 0x50, 0xA0, 0xE0, 0xF0]) | rng.choice([0, 1])
                words.append(encode(0xC3 | rng.choice([0x00, 0x18]), base, src, off, aop))
            else:
                off = rng.randrange(0, 64 - w + 1)
                if rng.random() < 0.4:
                    words.append(encode(0x62 | size, 1, 0, off, _imm(rng)))
                else:
                    words.append(encode(0x63 | size, 1, src, off))
            continue
        if pw_atomics and 0.55 <= q < 0.62:
            q = 0.5  # (no register-address loads)
        if q < 0.25:  # ST / STX into the window
            d = -rng.randrange(w, k + 1)
            base, off = (10, d) if c is None or rng.random() < 0.5 else (9, d + c)
            if rng.random() < 0.4:
                words.append(encode(0x62 | size, base, 0, off, _imm(rng)))
            else:
                words.append(encode(0x63 | size, base, src, off))
        elif q < 0.42:  # LDX from the window
            d = -rng.randrange(w, k + 1)
            base, off = (10, d) if c is None or rng.random() < 0.5 else (9, d + c)
            words.append(encode(0x61 | size, dst, base, off))
        elif q < 0.55:  # LDX from the packet
            words.append(encode(0x61 | size, dst, 1, rng.randrange(-2, 72)))
        elif q < 0.62:  # LDX around the window (512 - k - 8 .. 512 + 8): mostly through a
            r = rng.choice([3, 4, 5])                        # register the load-time dataflow
            if rng.random() < 0.75:                          # cannot resolve (r2 & 0 + c)
                words.append(encode(0xBF, r, 2, 0, 0))        # mov r, r2
                words.append(encode(0x57, r, 0, 0, 0))        # and r, 0
                words.append(encode(0x07, r, 0, 0, rng.randrange(512 - k - 8, 520)))
            else:                                            # else a constant address (whose
                words.append(encode(0xB7, r, 0, 0, rng.randrange(512 - k - 8, 520)))
                words.append(encode(0x0F, r, 1, 0, 0))        # overlap sends the batch to tier 1)
            words.append(encode(0x61 | size, dst, r, 0))
        elif q < 0.82:  # ALU (never on r9 / r10)
            cls = rng.choice([0x04, 0x07])
            op = rng.choice([0, 1, 2, 4, 5, 6, 7, 10, 11, 12])
            srcbit = rng.choice([0, 0x08])
            words.append(encode((op << 4) | srcbit | cls, dst, src, 0, _imm(rng)))
        elif q < 0.94:  # forward jumps
            cls = rng.choice([0x05, 0x06])
            op = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 10, 11, 12, 13])
            off = rng.randrange(0, max(1, n - len(words)) + 1)
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, off, _imm(rng)))
        else:
            words.append(encode(0x95))
    words.append(encode(0x95))
    return b"".join(words)


def gen_call_program(rng: random.Random, n: int | None = None, loops: bool = False) -> bytes:
    """Tier-0 programs with local calls (emu.rs:265-279: CALL jumps to t = pc + 1 + off and
    pushes t + 1, EXIT pops or stops): calls forward and backward, EXITs along the way, forward
    jumps (and with loops=True a few backward ones), packet loads and ALU ops. Some recurse (the
    frame stack grows until ST_CALLDEPTH or the budget), most reach a few frame stacks."""
    n = n or rng.randrange(6, 30)
    words: list[bytes] = []
    while len(words) < n:
        k = rng.random()
        pos = len(words)
        dst, src = rng.randrange(10), rng.randrange(10)
        if k < 0.16:  # CALL, mostly to a later instruction
            lo = -pos - 1 if rng.random() < 0.25 else 0
            words.append(encode(0x85, 0, 0, rng.randrange(lo, max(1, n - pos))))
        elif k < 0.27:
            words.append(encode(0x95))
        elif k < 0.55:
            cls = rng.choice([0x04, 0x07])
            op = rng.choice([0, 1, 2, 4, 5, 6, 7, 10, 11, 12])
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, 0, _imm(rng)))
        elif k < 0.70:
            cls = rng.choice([0x05, 0x06])
            op = rng.choice([1, 2, 3, 4, 5, 6, 7, 10, 11, 12, 13])
            off = rng.randrange(0, max(1, n - pos) + 1)
            if loops and rng.random() < 0.15:
                off = -rng.randrange(1, 4)
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, off, _imm(rng)))
        elif k < 0.85:
            size = rng.choice([0x00, 0x08, 0x10, 0x18])
            words.append(encode(0x61 | size, dst, 1, rng.randrange(0, 70)))
        else:
            words.append(encode(0xB7 | rng.choice([0, 0x08]), dst, src, 0, _imm(rng)))
    words.append(encode(0x95))
    return b"".join(words)


def gen_stack_loop_program(rng: random.Random, k: int = 32) -> bytes:
    """Stack-window programs with a loop (memory tier 0.5 on the loop kernel): before the loop, r9
    may point into the stack; the loop runs r7 = 0 .. N - 1 (N a constant or the packet length r2)
    over a body of stack stores / loads / atomics at r10 offsets, byte and word loads of the
    packet at r1 + r7 (+ c, some past the 64-byte window, some through registers aimed at the
    stack window: the store-forwarding overlay), and ALU ops; a forward exit from the body; a
    tail that folds stack bytes into r0."""
    sizes = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}
    words: list[bytes] = []
    words.append(encode(0xB7, 7, 0, 0, 0))                    # mov r7, 0
    words.append(encode(0x7A, 10, 0, -8, rng.choice([0, 1, 0x55])))  # stdw [r10-8], c
    c9 = rng.randrange(0, 9)
    words.append(encode(0xBF, 9, 10, 0, 0))                   # mov r9, r10
    words.append(encode(0x07, 9, 0, 0, -c9))                  # add r9, -c9
    body: list[bytes] = []
    nb = rng.randrange(3, 12)
    while len(body) < nb:
        q = rng.random()
        size = rng.choice(list(sizes))
        w = sizes[size]
        dst = rng.choice([0, 3, 4, 5, 6])
        src = rng.choice([0, 3, 4, 5, 6, 7])
        if q < 0.2:  # ST / STX into the window (r10 or r9)
            d = -rng.randrange(w, k + 1)
            base, off = (10, d) if rng.random() < 0.6 else (9, d + c9)
            if rng.random() < 0.3:
                body.append(encode(0x62 | size, base, 0, off, _imm(rng)))
            else:
                body.append(encode(0x63 | size, base, src, off))
        elif q < 0.35:  # LDX from the window
            d = -rng.randrange(w, k + 1)
            body.append(encode(0x61 | size, dst, 10, d))
        elif q < 0.55:  # packet bytes at r1 + r7 + c
            body.append(encode(0xBF, 4, 1, 0, 0))               # mov r4, r1
            body.append(encode(0x0F, 4, 7, 0, 0))               # add r4, r7
            body.append(encode(0x61 | size, dst if dst != 4 else 5, 4, rng.choice([0, 1, 3, 50, 61, 70, 200])))
        elif q < 0.62:  # a load aimed at the stack window through a register (overlay)
            body.append(encode(0xBF, 3, 7, 0, 0))               # mov r3, r7
            body.append(encode(0x57, 3, 0, 0, 7))               # and r3, 7
            body.append(encode(0x07, 3, 0, 0, 512 - k + rng.randrange(0, k)))
            body.append(encode(0x61 | size, dst if dst != 3 else 5, 3, 0))
        elif q < 0.70:  # a stack atomic
            d = -4 * rng.randrange(2, k // 4 + 1)
            aop = rng.choice([0x00, 0x40, 0x50, 0xA0, 0xE0, 0xF0]) | rng.choice([0, 1])
            body.append(encode(0xC3 | rng.choice([0x00, 0x18]), 10, rng.choice([3, 5, 6]), d, aop))
        elif q < 0.75:  # leave the loop early
            body.append(encode(0x55 | rng.choice([0, 0x08]), dst, src, 1 << 10, rng.randrange(0, 300)))
        else:  # ALU (never r7 / r9 / r10)
            op = rng.choice([0, 1, 2, 4, 5, 6, 7, 10, 11, 12])
            body.append(encode((op << 4) | rng.choice([0, 0x08]) | rng.choice([0x04, 0x07]), dst,
                               src, 0, _imm(rng)))
    # resolve the early exits (off placeholder 1 << 10) to the loop's end
    fixed = []
    for i, wd in enumerate(body):
        if wd[0] & 0x07 in (0x05, 0x06) and int.from_bytes(wd[2:4], "little") == 1 << 10:
            wd = wd[:2] + (len(body) - i - 1 + 2).to_bytes(2, "little") + wd[4:]
        fixed.append(wd)
    body = fixed
    words += body
    words.append(encode(0x07, 7, 0, 0, 1))                    # add r7, 1
    n = len(body) + 1
    if rng.random() < 0.5:
        words.append(encode(0xA5, 7, 0, -(n + 1), rng.randrange(1, 24)))  # jlt r7, N, loop
    else:
        words.append(encode(0xAD, 7, 2, -(n + 1)))             # jlt r7, r2, loop
    words.append(encode(0x79, 3, 10, -8))                      # ldxdw r3, [r10-8]
    words.append(encode(0x0F, 0, 3, 0, 0))                     # add r0, r3
    words.append(encode(0x71, 3, 10, -k))                      # ldxb r3, [r10-k]
    words.append(encode(0xAF, 0, 3, 0, 0))                     # xor r0, r3
    words.append(encode(0x95))
    return b"".join(words)


def gen_store_program(rng: random.Random, n: int | None = None) -> bytes:
    """Store-mode programs (register-address stores into the packet, host.cpp analyze_stack
    StackPlan::any_dyn; emu.rs:354-372): r8 = r1 + (a packet byte & m) + c -- a packet pointer the
    load-time dataflow cannot resolve -- and r7 = r8 + c2 (sometimes far past the image: faults);
    then ST/STX of every width through r8 / r7 (mostly inside the 64-byte header window, some
    past it or straddling its end: those lanes deoptimize to the general interpreter), loads
    through the same pointers (reading stored bytes back), constant-address loads and stores of
    the window, stack stores / loads / atomics at r10 - 8 .. r10 - 1, ALU and forward jumps; the
    registers folded into r0 at the end."""
    n = n or rng.randrange(8, 40)
    words: list[bytes] = [
        encode(0x71, 8, 1, 0, 0) if rng.random() < 0.2 else encode(0x71, 8, 1, rng.randrange(0, 64)),
        encode(0x57, 8, 0, 0, rng.choice([7, 15, 31, 63, 127])),      # and r8, m
        encode(0x07, 8, 0, 0, rng.randrange(0, 48)),                   # add r8, c
        encode(0x0F, 8, 1, 0, 0),                                      # add r8, r1
        encode(0xBF, 7, 8, 0, 0),                                      # mov r7, r8
        encode(0x07, 7, 0, 0, rng.choice([0, 2, 4, 8, 20, 40, 60, 1000, 1019, 2000])),
    ]
    regs = [0, 2, 3, 4, 5, 6]
    while len(words) < n:
        q = rng.random()
        size = rng.choice([0x00, 0x08, 0x10, 0x18])
        w = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}[size]
        dst, src = rng.choice(regs), rng.randrange(10)
        ptr = rng.choice([8, 8, 7])
        if q < 0.30:  # store through a pointer
            off = rng.choice([rng.randrange(-4, 64), rng.randrange(-4, 24), 60, 62, 70])
            if rng.random() < 0.35:
                words.append(encode(0x62 | size, ptr, 0, off, _imm(rng)))
            else:
                words.append(encode(0x63 | size, ptr, src, off))
        elif q < 0.48:  # load through a pointer
            words.append(encode(0x61 | size, dst, ptr, rng.choice([rng.randrange(-4, 64), 58, 61, 66])))
        elif q < 0.56:  # constant-address store into the window
            off = rng.randrange(0, 64 - w + 1)
            if rng.random() < 0.4:
                words.append(encode(0x62 | size, 1, 0, off, _imm(rng)))
            else:
                words.append(encode(0x63 | size, 1, src, off))
        elif q < 0.66:  # constant-address load (inside the window, or past it)
            off = rng.choice([rng.randrange(0, 64 - w + 1), rng.randrange(64, 90)])
            words.append(encode(0x61 | size, dst, 1, off))
        elif q < 0.72:  # the stack
            d = -rng.randrange(w, 9)
            if rng.random() < 0.5:
                words.append(encode(0x63 | size, 10, src, d))
            elif rng.random() < 0.5:
                words.append(encode(0x61 | size, dst, 10, d))
            else:
                words.append(encode(0xDB, 10, src, -8, 0x00))            # lock add [r10-8]
        elif q < 0.86:  # ALU (never on r1, r7 .. r10)
            cls = rng.choice([0x04, 0x07])
            op = rng.choice([0, 1, 2, 4, 5, 6, 7, 10, 11, 12])
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, 0, _imm(rng)))
        elif q < 0.97:  # forward jumps
            cls = rng.choice([0x05, 0x06])
            op = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 10, 11, 12, 13])
            off = rng.randrange(0, max(1, n - len(words)) + 1)
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, off, _imm(rng)))
        else:
            words.append(encode(0x95))
    for r in (3, 4, 5, 6):
        words.append(encode(0xAF, 0, r, 0, 0))                            # xor r0, r
    words.append(encode(0x95))
    return b"".join(words)


def gen_far_store_program(rng: random.Random, n: int | None = None) -> bytes:
    """Store-mode programs writing a 1500-byte frame's payload (jit.cpp's overflow image: image
    bytes [64, 2048) in 64-byte blocks filled on first use; emu.rs:354-372): r8 = r1 + (a packet
    byte << 2) + c (0 .. ~1400) and r7 = r8 + c2 -- pointers the load-time dataflow cannot resolve
    -- then stores of every width through them (some straddling 64-byte blocks), loads through
    them (stored bytes read back, other blocks read from the packet), loads at fixed payload
    offsets, window and stack accesses, ALU and forward jumps; the registers folded into r0."""
    n = n or rng.randrange(10, 40)
    words: list[bytes] = [
        encode(0x71, 8, 1, rng.randrange(0, 64)),                      # ldxb r8, [r1+k]
        encode(0x67, 8, 0, 0, rng.choice([0, 1, 2, 2, 2])),             # lsh r8, s
        encode(0x07, 8, 0, 0, rng.choice([0, 64, 100, 400, 700])),      # add r8, c
        encode(0x0F, 8, 1, 0, 0),                                       # add r8, r1
        encode(0xBF, 7, 8, 0, 0),                                       # mov r7, r8
        encode(0x07, 7, 0, 0, rng.choice([0, 4, 61, 64, 200, 630, 1100])),
    ]
    regs = [0, 2, 3, 4, 5, 6]
    while len(words) < n:
        q = rng.random()
        size = rng.choice([0x00, 0x08, 0x10, 0x18])
        w = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}[size]
        dst, src = rng.choice(regs), rng.randrange(10)
        ptr = rng.choice([8, 8, 7])
        if q < 0.32:  # store through a pointer
            off = rng.choice([rng.randrange(-4, 70), 60, 62, 63, 127, 125])
            if rng.random() < 0.35:
                words.append(encode(0x62 | size, ptr, 0, off, _imm(rng)))
            else:
                words.append(encode(0x63 | size, ptr, src, off))
        elif q < 0.52:  # load through a pointer
            words.append(encode(0x61 | size, dst, ptr, rng.choice([rng.randrange(-4, 70), 61, 63, 126])))
        elif q < 0.60:  # constant-address load past the window (the packet's payload)
            words.append(encode(0x61 | size, dst, 1, rng.choice([rng.randrange(64, 200), 1000, 1490])))
        elif q < 0.66:  # constant-address store / load in the window
            off = rng.randrange(0, 64 - w + 1)
            words.append(encode(0x63 | size, 1, src, off) if rng.random() < 0.5
                         else encode(0x61 | size, dst, 1, off))
        elif q < 0.72:  # the stack
            d = -rng.randrange(w, 9)
            words.append(encode(0x63 | size, 10, src, d) if rng.random() < 0.5
                         else encode(0x61 | size, dst, 10, d))
        elif q < 0.86:  # ALU (never on r1, r7 .. r10)
            cls = rng.choice([0x04, 0x07])
            op = rng.choice([0, 1, 2, 4, 5, 6, 7, 10, 11, 12])
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, 0, _imm(rng)))
        elif q < 0.97:  # forward jumps
            cls = rng.choice([0x05, 0x06])
            op = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 10, 11, 12, 13])
            off = rng.randrange(0, max(1, n - len(words)) + 1)
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src, off, _imm(rng)))
        else:
            words.append(encode(0x95))
    for r in (3, 4, 5, 6):
        words.append(encode(0xAF, 0, r, 0, 0))                            # xor r0, r
    words.append(encode(0x95))
    return b"".join(words)


def gen_slot_loop_program(rng: random.Random) -> bytes:
    """Loop programs that keep their accumulators in 8-byte stack slots, the way compiled C spills
    them (host.cpp promote_slots): `stdw [r10-8*k], c` before a byte loop over the packet
    (`ldxb rD, [r1 + rI]`, rI = start .. N, N = the packet length r2 or a constant), a body that
    reloads a slot, adds the byte (or xors / mixes it), stores it back -- sometimes through a
    second slot or with the accumulator register read after the store -- and a tail that folds
    the slots into r0. Some loops run through r2 + 16 (byte loads past the packet: not provable,
    no promotion)."""
    from ebpf_emu.asm import assemble

    nslots = rng.choice([1, 1, 2])
    start = rng.choice([0, 0, 1, 13])
    bound = rng.choice(["r2", "r2", "r2", "20", "r6"])
    acc = rng.choice(["r0", "r6", "r7"]) if bound != "r6" else rng.choice(["r0", "r7"])
    lines = [f"stdw [r10-{8 * (k + 1)}], {rng.choice([0, 0, 1, 0x55])}" for k in range(nslots)]
    if bound == "r6":
        lines += ["mov r6, r2", "add r6, 16"]
    lines += [f"mov r3, {start}", f"jge r3, {bound}, done", "loop:", "mov r4, r1", "add r4, r3",
              "ldxb r5, [r4+0]"]
    kind = rng.random()
    if kind < 0.6:  # the accumulator triple
        lines += [f"ldxdw {acc}, [r10-8]", f"add {acc}, r5", f"stxdw [r10-8], {acc}"]
    elif kind < 0.8:  # the register read again after the store (not foldable: rT live)
        lines += [f"ldxdw {acc}, [r10-8]", f"xor {acc}, r5", f"stxdw [r10-8], {acc}",
                  f"add {acc}, 1"]
    else:  # a mix
        lines += [f"ldxdw {acc}, [r10-8]", f"mul {acc}, 31", f"add {acc}, r5", f"stxdw [r10-8], {acc}"]
    if nslots == 2:
        lines += ["ldxdw r8, [r10-16]", "add r8, 1", "stxdw [r10-16], r8"]
    lines += ["add r3, 1", f"jlt r3, {bound}, loop", "done:", "ldxdw r0, [r10-8]"]
    if nslots == 2:
        lines += ["ldxdw r9, [r10-16]", "xor r0, r9"]
    lines += ["exit"]
    return assemble("\n".join(lines))


def gen_long_program(rng: random.Random, n: int, loops: bool = False, stack: bool = False,
                     store: bool = False) -> bytes:
    """Long tier-0 programs (hundreds to thousands of micro-ops, past the compiler's near-branch
    reach: jit.cpp far mode) that lanes actually run through: ALU ops on seeded registers, packet
    loads at r1 + 0..79 of every width, forward jumps over a few instructions, a rare early exit
    of some lanes;
    with loops=True also counted loops (r9 = 0 .. k) over a few instructions; with stack=True
    stores and loads of every width in the stack window [r10 - 32, r10) (memory tier 0.5); with
    store=True stores and loads through a packet pointer r8 = r1 + (a packet byte & 15) + c at
    offsets 0..99 (store mode: past byte 64 the overflow image, past 128 the deopt list). r0 folds
    the registers at the end."""
    words: list[bytes] = []
    for r in (0, 3, 4, 5, 6, 7, 8):
        v = rng.choice(EDGE) if rng.random() < 0.5 else rng.getrandbits(64)
        words.append(encode(0x18, r, 0, 0, v & 0xFFFFFFFF) + encode(0, 0, 0, 0, v >> 32))
    if stack:  # (the window's lowest store first: every later access lies inside [r10 - 32, r10))
        words.append(encode(0x7B, 10, 0, -32))                          # stxdw [r10-32], r0
    if store:
        words += [encode(0x71, 8, 1, rng.randrange(0, 64)),             # ldxb r8, [r1+c0]
                  encode(0x57, 8, 0, 0, 15), encode(0x07, 8, 0, 0, rng.randrange(0, 16)),
                  encode(0x0F, 8, 1, 0, 0)]                             # r8 = r1 + (b & 15) + c
    regs = [0, 3, 4, 5, 6, 7] if store else [0, 3, 4, 5, 6, 7, 8]
    while len(words) < n:
        q = rng.random()
        dst, src = rng.choice(regs), rng.choice([0, 2, 3, 4, 5, 6, 7, 8])
        if q < 0.08 and store:
            size = rng.choice([0x00, 0x08, 0x10, 0x18])
            off = rng.randrange(0, 100)
            k = rng.random()
            if k < 0.45:
                words.append(encode(0x63 | size, 8, src, off))           # stx [r8 + off], src
            elif k < 0.65:
                words.append(encode(0x62 | size, 8, 0, off, _imm(rng)))  # st [r8 + off], imm
            else:
                words.append(encode(0x61 | size, dst, 8, off))           # ldx dst, [r8 + off]
        elif q < 0.55:
            cls = rng.choice([0x04, 0x07])
            op = rng.choice([0, 1, 2, 4, 5, 6, 7, 10, 11, 12] * 4 + [3, 9, 13])
            srcbit = rng.choice([0, 0x08])
            imm = rng.choice([16, 32, 64]) if op == 13 else _imm(rng)
            words.append(encode((op << 4) | (0 if op == 13 else srcbit) | cls, dst,
                                0 if op == 13 else src, 0, imm))
        elif q < 0.75:
            size = rng.choice([0x00, 0x08, 0x10, 0x18])
            off = rng.randrange(0, 80)
            if store:  # (store mode: no constant-address load straddles byte 64, analyze_stack)
                w = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}[size]
                off = off if off >= 64 or off + w <= 64 else 64 - w
            words.append(encode(0x61 | size, dst, 1, off))
        elif q < 0.93:
            cls = rng.choice([0x05, 0x06])
            op = rng.choice([1, 2, 3, 4, 5, 6, 7, 10, 11, 12, 13])
            words.append(encode((op << 4) | rng.choice([0, 0x08]) | cls, dst, src,
                                rng.randrange(0, 7), _imm(rng)))
        elif q < 0.96 and stack:
            size = rng.choice([0x00, 0x08, 0x10, 0x18])
            w = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}[size]
            d = -w * rng.randrange(1, 32 // w + 1)
            k = rng.random()
            if k < 0.35:
                words.append(encode(0x63 | size, 10, src, d))           # stx [r10 + d], src
            elif k < 0.5:
                words.append(encode(0x62 | size, 10, 0, d, _imm(rng)))  # st [r10 + d], imm
            else:
                words.append(encode(0x61 | size, dst, 10, d))           # ldx dst, [r10 + d]
        elif q < 0.96 and loops:
            body = [encode(0x07 | (rng.choice([0, 1, 2, 10, 12]) << 4), rng.choice([3, 4, 5, 6]),
                           0, 0, _imm(rng)) for _ in range(rng.randrange(1, 5))]
            words.append(encode(0xB7, 9, 0, 0, 0))                      # mov r9, 0
            words += body
            words.append(encode(0x07, 9, 0, 0, 1))                      # add r9, 1
            words.append(encode(0xA5, 9, 0, -(len(body) + 2), rng.randrange(1, 12)))  # jlt r9, k
        elif q < 0.962:  # an exit for the lanes with dst == imm (the rest stays reachable)
            words += [encode(0x55, dst, 0, 1, rng.choice([0, 1, 2, 7, 0xFF])), encode(0x95)]
        else:
            words.append(encode(0xB7 | rng.choice([0, 0x08]), dst, src, 0, _imm(rng)))
    for r in (3, 4, 5, 6, 7, 8):
        words.append(encode(0xAF, 0, r, 0, 0))                          # xor r0, r
    words.append(encode(0x95))
    return b"".join(words)
