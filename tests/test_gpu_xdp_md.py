"""The xdp_md calling convention (EBPF_BATCH_XDP_MD; xdp.rs:16-20): every
packet's image is [u32 data = 8][u32 data_end = 8 + len][packet], r1 = 0 points at the ctx and
r2 = 8 + len. Checked against the oracle run on exactly those ctx-prefixed images -- the bytes the
reference's main.rs would be handed -- for a standard bounds-checked XDP parser, a loop program,
both input layouts and images longer than the memory (ST_BADPKT)."""
import random
import struct

import numpy as np
import pytest

from test_gpu_parity import _stage

pytestmark = pytest.mark.gpu

# a verifier-style XDP program: ctx->data / ctx->data_end, explicit bounds checks, then the parse
XDP_PARSE = """
    ldxw r2, [r1+0]           # ctx->data
    ldxw r3, [r1+4]           # ctx->data_end
    mov r0, 2                 # XDP_PASS
    mov r4, r2
    add r4, 14
    jgt r4, r3, out           # no Ethernet header
    ldxh r5, [r2+12]
    jne r5, 0x0008, out       # not IPv4
    mov r4, r2
    add r4, 34
    jgt r4, r3, out           # no IPv4 header
    ldxb r6, [r2+23]
    jne r6, 17, out           # not UDP
    mov r0, 1                 # XDP_DROP
out:
    exit
"""

# loop over the packet bytes between data and data_end
XDP_SUM = """
    ldxw r2, [r1+0]
    ldxw r3, [r1+4]
    mov r0, 0
loop:
    jge r2, r3, done
    ldxb r5, [r2+0]
    add r0, r5
    add r2, 1
    ja loop
done:
    exit
"""


# the loop bound reloaded from the ctx every iteration (a compiled xdp_md loop program's ctx
# loads, jit.cpp ctx_load, inside the loop)
XDP_SUM_RELOAD = """
    ldxw r2, [r1+0]
    mov r0, 0
loop:
    ldxw r3, [r1+4]
    jge r2, r3, done
    ldxb r5, [r2+0]
    add r0, r5
    add r2, 1
    ja loop
done:
    exit
"""

# the bound reloaded every iteration through a saved ctx pointer (compilers keep ctx in r6: a
# copy of r1, jit.cpp ctx_load's register set) -- in place, not staged
XDP_SUM_CTX_SAVED = """
    mov r6, r1
    ldxw r2, [r6+0]
    mov32 r7, r6
    mov r0, 0
loop:
    ldxw r3, [r7+4]
    jge r2, r3, done
    ldxb r5, [r2+0]
    add r0, r5
    add r2, 1
    ja loop
done:
    exit
"""

# a ctx-shaped load that is not the ctx on every path (r1 moved on one of them): compiled as a
# load, not as the ctx's data_end
XDP_R1_MOVED = """
    ldxw r2, [r1+0]
    ldxw r3, [r1+4]
    mov r0, 0
    ldxb r4, [r2+0]
    jeq r4, 0, skip
    add r1, 4
skip:
    ldxw r6, [r1+4]
    add r0, r6
loop:
    jge r2, r3, done
    ldxb r5, [r2+0]
    add r0, r5
    add r2, 1
    ja loop
done:
    exit
"""


def _images(pkts):
    return [struct.pack("<II", 8, 8 + len(p)) + p for p in pkts]


@pytest.mark.parametrize("layout", [dict(), dict(offsets_layout=True, misalign=3)])
@pytest.mark.parametrize("src", [XDP_PARSE, XDP_SUM, XDP_SUM_RELOAD, XDP_R1_MOVED])
def test_xdp_md_images_match_oracle(cuda, oracle_mod, layout, src):
    import torch

    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    rng = random.Random(5)
    pkts = []
    for _ in range(300):
        n = rng.choice([0, 10, 14, 33, 34, 60, 64, 100, 1010, 1016, 1017, 1400])
        p = bytearray(rng.getrandbits(8) for _ in range(n))
        if n >= 24 and rng.random() < 0.7:
            p[12:14] = b"\x08\x00"
            p[23] = rng.choice([6, 17])
        pkts.append(bytes(p))
    img = assemble(src)
    prog = Program(img)
    frames, kw = _stage(pkts, cuda, **layout)
    res = prog.run(frames, r0=True, status=True, regs=True, mem=True, xdp_md=True,
                   counters=torch.zeros(8, dtype=torch.int64, device=cuda), **kw)
    torch.cuda.synchronize()
    status = res.status.cpu().numpy()
    regs = res.regs.cpu().numpy().view(np.uint64)
    mem = res.mem.cpu().numpy()
    op = oracle_mod.Program(img)
    for i, im in enumerate(_images(pkts)):
        st, oregs, omem, _ = op.run_full(im, 1024, 512, 20000)
        assert status[i] == st, (i, len(pkts[i]))
        if st == 0:
            assert [int(v) for v in regs[i]] == oregs, i
            assert bytes(mem[i]) == omem, i
    assert (status == 7).sum() == sum(len(p) + 8 > 1024 for p in pkts)  # ST_BADPKT
    prog.close()


def _xdp_packets(rng, n, lens=(0, 1, 7, 10, 14, 33, 34, 60, 64, 100, 1010, 1016, 1017, 1400)):
    pkts = []
    for _ in range(n):
        p = bytearray(rng.getrandbits(8) for _ in range(rng.choice(lens)))
        if len(p) >= 24 and rng.random() < 0.7:
            p[12:14] = b"\x08\x00"
            p[23] = rng.choice([6, 17])
        pkts.append(bytes(p))
    return pkts


@pytest.mark.parametrize("layout", [dict(), dict(offsets_layout=True, align=16),
                                    dict(offsets_layout=True, misalign=3)])
@pytest.mark.parametrize("src", [XDP_PARSE, XDP_SUM, XDP_SUM_RELOAD, XDP_R1_MOVED])
def test_xdp_md_production_outputs(cuda, oracle_mod, layout, src):
    """The outputs a production caller asks for, no registers and no image: a verdict + counters
    launch, then an r0 + status launch -- the compiled kernels' liveness-pruned register init
    and output-free epilogue -- per packet against the oracle on the ctx-prefixed images
    (main.rs:14-43 handed [xdp_md][packet], xdp.rs:16-20), short packets and ST_BADPKT included,
    with the retired-instruction counter."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    rng = random.Random(17)
    pkts = _xdp_packets(rng, 333)
    img = assemble(src)
    prog = Program(img)
    frames, kw = _stage(pkts, cuda, **layout)
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    v = prog.run(frames, verdict=True, counters=cnt, xdp_md=True, **kw)
    rs = prog.run(frames, verdict=False, r0=True, status=True, xdp_md=True, **kw)
    torch.cuda.synchronize()
    verdict = v.verdict.cpu().numpy()
    r0 = rs.r0.cpu().numpy().view(np.uint64)
    status = rs.status.cpu().numpy()
    want = np.zeros(8, dtype=np.uint64)
    op = oracle_mod.Program(img)
    for i, im in enumerate(_images(pkts)):
        st, or0, steps = op.run_packet(im, 1024, 512, 1 << 22)
        assert status[i] == st, (i, len(pkts[i]))
        if st == 0:
            assert int(r0[i]) == or0, i
            assert verdict[i] == (or0 if or0 < 5 else 0xFE), i
            want[or0 if or0 < 5 else 5] += 1
        else:
            assert verdict[i] == 0xFF, i
            want[6] += 1
        want[7] += steps
    assert list(cnt.cpu().numpy().view(np.uint64)) == list(want)
    assert (status == 7).sum() == sum(len(p) + 8 > 1024 for p in pkts)  # ST_BADPKT
    prog.close()


# ctx and packet bytes mixed in one access, reads past the 64-byte window and across its end, a
# register address from r2 (= data_end in the main.rs layout of an xdp_md image)
XDP_CTX_MIX = """
    ldxdw r3, [r1+0]          # data | data_end << 32
    ldxdw r4, [r1+4]          # data_end | packet bytes 0..3 << 32
    ldxw r5, [r1+6]           # ctx and packet bytes in one word
    mov r0, r3
    xor r0, r4
    add r0, r5
    ldxb r6, [r1+70]          # packet byte 62: past the window
    add r0, r6
    ldxw r7, [r1+60]          # across the window's end
    xor r0, r7
    mov r8, r1
    add r8, r2
    ldxb r9, [r8-1]           # the last packet byte, register address
    lsh r9, 8
    add r0, r9
    ldxh r9, [r3+4]           # packet bytes 4..5 through r3 = data (its low word)
    xor r0, r9
    exit
"""


def _route(prog, frames, kw, **extra):
    return prog.batch_kernel(prog.make_batch(frames, xdp_md=True, **kw, **extra))


@pytest.mark.parametrize("stride,mem", [(64, 1024), (96, 1024), (64, 72), (64, 71), (128, 100)])
def test_xdp_md_fixed_slots_in_place(cuda, oracle_mod, stride, mem):
    """Fixed slots (no lengths: every packet `stride` bytes): the compiled fixed-slot kernel runs
    the xdp_md batch in place (the ctx synthesised in its LDS window, no staging kernel); every
    output against the oracle on the ctx-prefixed images, and against the staged general
    interpreter. Images of exactly mem_size bytes, and one byte past it (ST_BADPKT)."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    n = 777
    buf = W.frames_fixed(n, stride, 3)
    frames = torch.from_numpy(buf).to(cuda)
    pkts = [bytes(buf[i * stride:(i + 1) * stride]) for i in range(n)]
    for src in (XDP_PARSE, W.FIVE_TUPLE_XDP, XDP_CTX_MIX):
        img = assemble(src)
        prog = Program(img)
        assert prog.compile()
        assert _route(prog, frames, dict(n=n, stride=stride), mem_size=mem) == \
            _lib.EBPF_KERNEL_JIT_FIXED
        cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
        v = prog.run(frames, n=n, stride=stride, mem_size=mem, counters=cnt, xdp_md=True)
        rs = prog.run(frames, n=n, stride=stride, mem_size=mem, verdict=False, r0=True,
                      status=True, xdp_md=True)
        full = prog.run(frames, n=n, stride=stride, mem_size=mem, r0=True, status=True,
                        regs=True, xdp_md=True)
        gen = prog.run(frames, n=n, stride=stride, mem_size=mem, r0=True, status=True,
                       regs=True, xdp_md=True, generic=True)
        torch.cuda.synchronize()
        r0, st, ocnt = oracle_mod.Program(img).run_batch(buf, n, stride=stride, mem_size=mem,
                                                         xdp_md=True, threads=4)
        assert np.array_equal(rs.status.cpu().numpy(), st), src[:30]
        ok = st == 0
        assert np.array_equal(rs.r0.cpu().numpy().view(np.uint64)[ok], r0[ok])
        want_v = np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8)
        assert np.array_equal(v.verdict.cpu().numpy(), want_v)
        assert list(cnt.cpu().numpy().view(np.uint64)) == list(ocnt)
        for k in ("r0", "status", "regs"):
            assert torch.equal(getattr(full, k), getattr(gen, k)), (k, src[:30])
        for i in range(0, n, 97):  # every register of a sample against the oracle
            ost, oregs, _, _ = oracle_mod.Program(img).run_full(
                struct.pack("<II", 8, 8 + stride) + pkts[i], mem, 512, 1 << 22)
            assert ost == st[i]
            if ost == 0:
                assert [int(x) for x in full.regs[i].cpu().numpy().view(np.uint64)] == oregs
        prog.close()


@pytest.mark.parametrize("layout", [dict(), dict(offsets_layout=True, align=16),
                                    dict(offsets_layout=True, misalign=3)])
def test_xdp_md_var_in_place(cuda, oracle_mod, layout):
    """Offsets + lens and stride + lens layouts: the compiled var kernel runs the batch in place
    (window shifted in LDS by the C++ prologue), the final images included; against the oracle
    and the staged general interpreter."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu.asm import assemble

    rng = random.Random(23)
    pkts = _xdp_packets(rng, 260)
    for src in (XDP_PARSE, XDP_CTX_MIX):
        img = assemble(src)
        prog = Program(img)
        frames, kw = _stage(pkts, cuda, **layout)
        # (without final images: the var tile loop, on stride + lens for 16-byte aligned slots)
        assert _route(prog, frames, kw) in (_lib.EBPF_KERNEL_JIT_VARL, _lib.EBPF_KERNEL_JIT_VAR)
        full = prog.run(frames, r0=True, status=True, regs=True, mem=True, xdp_md=True, **kw)
        gen = prog.run(frames, r0=True, status=True, regs=True, mem=True, xdp_md=True,
                       generic=True, **kw)
        torch.cuda.synchronize()
        for k in ("r0", "status", "regs"):
            assert torch.equal(getattr(full, k), getattr(gen, k)), (k, src[:30], layout)
        # (the final image of a packet too long for it, ST_BADPKT, is not defined: the reference
        # panics before it has one, main.rs:20-21)
        ok = full.status == 0
        assert torch.equal(full.mem[ok], gen.mem[ok]), (src[:30], layout)
        op = oracle_mod.Program(img)
        status = full.status.cpu().numpy()
        for i, im in enumerate(_images(pkts)):
            st, oregs, omem, _ = op.run_full(im, 1024, 512, 1 << 22)
            assert status[i] == st, i
            if st == 0:
                assert [int(x) for x in full.regs[i].cpu().numpy().view(np.uint64)] == oregs
                assert bytes(full.mem[i].cpu().numpy()) == omem
        prog.close()


# the sum in words, halves and bytes (loads of every width, none at a fixed window position)
XDP_SUM_WIDE = """
    ldxw r2, [r1+0]
    ldxw r3, [r1+4]
    mov r0, 0
    mov r4, r2
    add r4, 4
loop4:
    jgt r4, r3, tail
    ldxw r5, [r4-4]
    add r0, r5
    ldxh r6, [r4-2]
    xor r0, r6
    add r4, 4
    ja loop4
tail:
    mov r2, r4
    sub r2, 4
loop1:
    jge r2, r3, done
    ldxb r5, [r2+0]
    add r0, r5
    add r2, 1
    ja loop1
done:
    exit
"""


@pytest.mark.parametrize("layout", [dict(), dict(offsets_layout=True, align=16),
                                    dict(offsets_layout=True, misalign=3)])
def test_xdp_md_loop_programs_in_place(cuda, oracle_mod, layout):
    """Loop programs whose every packet load is proven past the ctx run the xdp_md batch in place
    (no staging kernel): variant 6, the program rebased -- packet loads 8 bytes lower, the batch
    run as the main.rs layout over the packets with mem_size - 8, r2 and the ctx's data_end 8 + LEN
    (jit.cpp Compiler::xdp_rebase). Status, r0, every register, verdicts and counters against the
    oracle on the ctx-prefixed images (xdp.rs:16-20), short packets, ST_BADPKT and a step budget
    that binds (the exact copy) included. A program with a load that may read the ctx, and a batch
    asking for the final images, stay staged."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    rng = random.Random(29)
    pkts = _xdp_packets(rng, 400)
    frames, kw = _stage(pkts, cuda, **layout)
    for src in (XDP_SUM, XDP_SUM_RELOAD, XDP_SUM_CTX_SAVED, XDP_SUM_WIDE, W.CHECKSUM_XDP):
        img = assemble(src) if isinstance(src, str) else src
        prog = Program(img)
        assert prog.compile()
        b = prog.make_batch(frames, xdp_md=True, **kw)
        assert prog.batch_kernel(b) == _lib.EBPF_KERNEL_JIT_LOOP
        assert not prog.batch_staged(b), src
        op = oracle_mod.Program(img)
        for steps in (1 << 22, 50):
            cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
            res = prog.run(frames, r0=True, status=True, regs=True, counters=cnt, xdp_md=True,
                           max_steps=steps, **kw)
            torch.cuda.synchronize()
            status = res.status.cpu().numpy()
            regs = res.regs.cpu().numpy().view(np.uint64)
            verdict = res.verdict.cpu().numpy()
            want = np.zeros(8, dtype=np.uint64)
            for i, im in enumerate(_images(pkts)):
                st, oregs, _, nst = op.run_full(im, 1024, 512, steps)
                want[7] += nst
                assert status[i] == st, (i, len(pkts[i]), steps)
                if st == 0:
                    assert [int(x) for x in regs[i]] == oregs, (i, steps)
                    assert verdict[i] == (oregs[0] if oregs[0] < 5 else 0xFE)
                    want[oregs[0] if oregs[0] < 5 else 5] += 1
                else:
                    assert verdict[i] == 0xFF
                    want[6] += 1
            assert list(cnt.cpu().numpy().view(np.uint64)) == list(want), steps
            assert (status == 7).sum() == sum(len(p) + 8 > 1024 for p in pkts)
            if steps == 50:
                assert (status == 5).sum() > 0  # (ST_STEPS: the budget bound)
        # final images: the staged images (they hold the ctx)
        o = _lib.BatchOut()
        o.mem = 16
        assert prog.batch_staged(b, o)
        prog.close()
    prog = Program(assemble(XDP_R1_MOVED))  # (ldxw r6, [r1+4] may read the ctx's data_end)
    assert prog.compile() and prog.batch_staged(prog.make_batch(frames, xdp_md=True, **kw))
    prog.close()


def test_xdp_md_checksum_loop_full_size(cuda):
    """The per-byte checksum as a standard XDP program (workloads.CHECKSUM_XDP: the sum over
    ctx->data .. ctx->data_end, a loop program run in place, rebased) over a 256 Ki slice of config 5's mixed 64/1500-byte frames with 2048-byte
    images: the same verdicts and verdict counters as the plain checksum (CHECKSUM, main.rs
    layout) on the same packets, which test_workload_golden_full_size pins to the oracle."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    n = 1 << 18
    buf, offs, lens = W.frames_mixed(n)
    frames = torch.from_numpy(buf).to(cuda)
    kw = dict(n=n, offsets=torch.from_numpy(offs.view(np.int32)).to(cuda),
              lens=torch.from_numpy(lens.view(np.int16)).to(cuda), mem_size=2048, r10=2048)
    out = {}
    for name, xdp in (("checksum", False), ("checksum_xdp", True)):
        prog = Program(W.program(name))
        if xdp:
            assert not prog.batch_staged(prog.make_batch(frames, xdp_md=True, **kw))
        cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
        res = prog.run(frames, counters=cnt, xdp_md=xdp, **kw)
        torch.cuda.synchronize()
        out[name] = (res.verdict.cpu().numpy(), cnt.cpu().numpy().view(np.uint64))
        prog.close()
    assert np.array_equal(out["checksum"][0], out["checksum_xdp"][0])
    assert list(out["checksum"][1][:7]) == list(out["checksum_xdp"][1][:7])
    assert (out["checksum"][0] == 1).sum() > 1000 and (out["checksum"][0] == 2).sum() > 1000


def _xdp_loop_program(rng):
    """A random xdp_md loop over data .. data_end: the pointer itself compared with data_end
    (shape A) or an end pointer r4 = p + K (shape B); loads of every width at offsets inside the
    step's span; r0 mixed with xor / add / shifts; data_end optionally reloaded from the ctx."""
    w, suffix = rng.choice([(1, "b"), (2, "h"), (4, "w"), (8, "dw")])
    reload = rng.random() < 0.3
    mix = rng.choice(["xor r0, r5", "add r0, r5", "lsh r0, 1\n    xor r0, r5", "add r0, r5\n    rsh r0, 3"])
    lines = ["ldxw r2, [r1+0]", "ldxw r3, [r1+4]", f"mov r0, {rng.randrange(256)}"]
    if rng.random() < 0.5:
        step = rng.randrange(1, 9)
        off = rng.randrange(0, 8)
        lines += ["loop:"] + (["ldxw r3, [r1+4]"] if reload else []) + [
            "jge r2, r3, done", f"ldx{suffix} r5, [r2+{off}]", mix, f"add r2, {step}", "ja loop"]
    else:
        K = rng.randrange(w, 17)
        step = rng.randrange(1, K + 1)
        off = rng.randrange(0, K - w + 1)
        lines += ["mov r4, r2", f"add r4, {K}", "loop:"] + (["ldxw r3, [r1+4]"] if reload else []) + [
            "jgt r4, r3, done", f"ldx{suffix} r5, [r4-{K - off}]", mix, f"add r4, {step}", "ja loop"]
    lines += ["done:", "exit"]
    return "\n".join("    " + ln if not ln.endswith(":") else ln for ln in lines) + "\n"


@pytest.mark.parametrize("seed", range(3))
def test_xdp_md_loop_fuzz_in_place(cuda, oracle_mod, seed):
    """Random xdp_md loop programs (_xdp_loop_program) on an offsets + lens batch of short and
    long packets: run in place (rebased) where the range analysis proves every load past the ctx,
    else staged; either way status, r0 and every register against the oracle on the ctx-prefixed
    images (xdp.rs:16-20), with a budget that binds on the long packets too. Most programs must
    run in place."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    rng = random.Random(1000 + seed)
    pkts = _xdp_packets(rng, 200)
    frames, kw = _stage(pkts, cuda, offsets_layout=True, align=16 if seed != 2 else 1,
                        misalign=0 if seed != 2 else 5)
    in_place = 0
    for k in range(10):
        src = _xdp_loop_program(rng)
        img = assemble(src)
        prog = Program(img)
        assert prog.compile(), src
        in_place += not prog.batch_staged(prog.make_batch(frames, xdp_md=True, **kw))
        op = oracle_mod.Program(img)
        for steps in (1 << 22, 300):
            res = prog.run(frames, r0=True, status=True, regs=True, xdp_md=True, max_steps=steps,
                           **kw)
            torch.cuda.synchronize()
            status = res.status.cpu().numpy()
            regs = res.regs.cpu().numpy().view(np.uint64)
            for i, im in enumerate(_images(pkts)):
                st, oregs, _, _ = op.run_full(im, 1024, 512, steps)
                assert status[i] == st, (src, i, len(pkts[i]), steps)
                if st == 0:
                    assert [int(x) for x in regs[i]] == oregs, (src, i, steps)
        prog.close()
    assert in_place >= 6, in_place


@pytest.mark.parametrize("r1", [8, 4, 0])
def test_xdp_md_loop_init_regs(cuda, oracle_mod, r1):
    """Caller-set registers (batch.init_regs, emu.rs:14-17) on an xdp_md batch of loop programs:
    with r1 != 0 the program's `ldxw rX, [r1+0/4]` are packet loads, not the ctx's data /
    data_end, so neither the staged-ctx variant (5, which compiles them as the ctx's constants)
    nor the rebased one (6) may run. Every packet's status / r0 / registers against the oracle on
    the ctx-prefixed images with the same registers, and against the general interpreter.
    The packets' first 8 bytes are in-image offsets, so with r1 = 8 the loops run over them."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    rng = random.Random(77 + r1)
    pkts = []
    for p in _xdp_packets(rng, 240, lens=(8, 9, 16, 40, 64, 100, 600)):
        p = bytearray(p)
        k = rng.randrange(0, len(p) + 1)
        p[0:4] = struct.pack("<I", 8 + k)
        p[4:8] = struct.pack("<I", 8 + len(p) - rng.randrange(0, 3))
        pkts.append(bytes(p))
    regs0 = [0, r1, 0, 0, 0, 0, 0, 0, 0, 0, 512]
    ir = torch.tensor(np.array(regs0, dtype=np.uint64).view(np.int64), device=cuda)
    frames, kw = _stage(pkts, cuda, offsets_layout=True, align=16)
    for src in (XDP_SUM, XDP_SUM_RELOAD, XDP_SUM_WIDE, W_CHECKSUM_XDP()):
        img = assemble(src) if isinstance(src, str) else src
        prog = Program(img)
        op = oracle_mod.Program(img)
        for steps in (1 << 22, 200):
            got = prog.run(frames, r0=True, status=True, regs=True, xdp_md=True, init_regs=ir,
                           max_steps=steps, **kw)
            gen = prog.run(frames, r0=True, status=True, regs=True, xdp_md=True, init_regs=ir,
                           max_steps=steps, generic=True, **kw)
            prod = prog.run(frames, r0=True, status=True, xdp_md=True, init_regs=ir,
                            max_steps=steps, **kw)
            torch.cuda.synchronize()
            for k in ("r0", "status", "regs"):
                assert torch.equal(getattr(got, k), getattr(gen, k)), (k, r1, steps)
            assert torch.equal(prod.status, got.status) and torch.equal(prod.r0, got.r0)
            status = got.status.cpu().numpy()
            regs = got.regs.cpu().numpy().view(np.uint64)
            for i, im in enumerate(_images(pkts)):
                st, oregs, _, _ = op.run_full(im, 1024, 512, steps, init_regs=regs0)
                assert status[i] == st, (i, r1, steps)
                if st == 0:
                    assert [int(x) for x in regs[i]] == oregs, (i, r1, steps)
        prog.close()


def W_CHECKSUM_XDP():
    from ebpf_emu import workloads as W

    return W.program("checksum_xdp")
