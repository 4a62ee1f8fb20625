"""Memory tier 0.5 (stack-window programs, host.cpp analyze_stack, jit.cpp stack_* / pw_store):
programs whose memory writes are ST/STX/ATOMIC at r10 + c, or ST/STX into the packet's header
window at constant addresses, keep the stack window [r10 - k, r10) in VGPRs of the compiled
fixed-slot kernel (and the stored window bytes in its preloaded window registers) instead of
running on the general interpreter with per-packet images.

CPU: the load-time analysis on directed programs (which are stack-window programs and how large
their window is), and every eligible fuzzed program compiles and assembles.
GPU: the compiled stack-window kernel against the general interpreter (EBPF_BATCH_GENERIC, tier 1)
and the oracle on the same batch -- status, r0, every register, verdicts and counters -- and the
launches that must fall back to the general interpreter (window over the packet, image output,
other layouts, init_regs), each still equal to the oracle. Reference: emu.rs:354-372 (ST/STX),
emu.rs:341-349 (LDX), main.rs:28-31 (r10 = 512)."""
import random
import zlib

import numpy as np
import pytest

from fuzzgen import gen_packet, gen_stack_loop_program, gen_stack_program

STEPS = 20000

DIRECTED = [
    ("stxdw [r10-8], r1\nexit", 8),
    ("stb [r10-1], 1\nexit", 4),                                   # rounded up to a dword
    ("mov r2, r10\nadd r2, -16\nstxw [r2+4], r3\nexit", 12),      # through a copy of r10
    ("mov r2, r10\nsub r2, 20\nsth [r2+0], 7\nexit", 20),
    ("stxdw [r10-64], r1\nexit", 64),
    ("stxdw [r10-72], r1\nexit", 0),                               # past kStackMax
    ("stxw [r10-2], r1\nexit", 0),                                 # crosses r10
    ("stxw [r1+0], r2\nexit", 4),                                  # a packet-window store
    ("stxw [r1+60], r2\nldxw r0, [r1+60]\nexit", 4),              # stored, then read back
    ("stxw [r1+62], r2\nexit", 0),                                 # crosses the window's end
    ("stxw [r1+8], r2\nmov r3, r2\nldxb r0, [r3+0]\nexit", 0),    # + a register-address load
    ("stxw [r1+8], r2\nldxw r0, [r1+62]\nexit", 0),               # + a load across byte 64
    ("stxw [r1+8], r2\nldxw r0, [r10-8]\nexit", 0),               # + a load outside the window
    ("mov r3, r2\nstxw [r3+0], r2\nexit", 4),                     # through an unknown pointer:
                                                                   # store mode (test_store_mode.py)
    ("jeq r2, 60, +2\nmov r3, r10\nja +1\nmov r3, r1\nstxb [r3-4], r0\nexit", 4),  # join differs:
                                                                   # store mode
    ("jeq r2, 60, +2\nmov r3, r10\nja +1\nmov r3, r10\nstxb [r3-4], r0\nexit", 4),  # join agrees
    ("stxdw [r10-8], r1\nldxw r0, [r10-10]\nexit", 0),             # a load straddling the edge
    ("stxdw [r10-8], r1\nldxw r0, [r10-16]\nexit", 8),             # a load below the window
    ("stxdw [r10-8], r1\nlock add [r10-16], r2\nexit", 16),        # a stack atomic (8 bytes)
    ("lock fetch add32 [r10-8], r2\nexit", 8),
    ("lock add [r10-6], r2\nexit", 0),                             # misaligned atomic
    ("lock add [r1+8], r2\nexit", 0),                              # an atomic on the packet
    ("stxdw [r10-8], r1\ncall 0\nexit", 8),                        # calls (flatten_calls)
    ("mov r0, 0\nstxb [r10-1], r0\nadd r0, 1\njlt r0, 5, -3\nexit", 4),  # a loop (loop kernel)
    ("mov r0, 0\nstxb [r1+3], r0\nadd r0, 1\njlt r0, 5, -3\nexit", 0),  # + packet store
    ("mov32 r2, r10\nstxb [r2-1], r0\nexit", 4),                   # a truncated pointer: store mode
    ("mov r0, 1\nexit", 0),                                        # no store: tier 0
]


def test_stack_analysis_directed(product_lib):
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    for src, k in DIRECTED:
        p = Program(assemble(src))
        assert p.stack_window == k, (src, p.stack_window)
        if k:
            assert p.tier == 1 and p.compile(), src
        p.close()


def test_stack_programs_compile():
    """Every eligible random stack program compiles and assembles (on the CPU); its code keeps no
    interpreter machinery and writes the window registers."""
    from ebpf_emu import Program

    rng = random.Random(2024)
    n_ok = 0
    for it in range(350):
        img = gen_stack_program(rng, pw_atomics=it >= 250)
        try:
            p = Program(img)
        except Exception:
            continue
        if p.stack_window:
            assert p.compile(), img.hex()
            text = p.jit_asm(1)
            body = text[text.index("; compiled eBPF program"):]
            body = body[:body.index(".Ldone")]
            for word in ("s_set_gpr_idx", "s_setpc", "s_load_dwordx16", "s_ff1"):
                assert word not in body, word
            assert "; stack window:" in body
            n_ok += 1
        p.close()
    assert n_ok >= 150


# ---------------------------------------------------------------------------------------------
def _fixed_frames(pkts, stride, dev):
    import torch

    buf = np.zeros(len(pkts) * stride, dtype=np.uint8)
    for i, p in enumerate(pkts):
        buf[i * stride:i * stride + len(p)] = np.frombuffer(p, dtype=np.uint8)
    return torch.tensor(buf, device=dev)


def _run(img, frames, n, dev, kernel=None, generic=False, **kw):
    import torch

    from ebpf_emu import Program, _lib

    prog = Program(img)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    mem = kw.pop("mem", False)
    b = prog.make_batch(frames, n=n, generic=generic, max_steps=STEPS, **kw)
    o = _lib.BatchOut()
    if mem:
        o.mem = 1
    got_kernel = prog.batch_kernel(b, o, dev.index or 0)
    if kernel is not None:
        assert got_kernel == kernel, (_lib.KERNEL_NAMES[got_kernel], img.hex())
    res = prog.run(frames, n=n, max_steps=STEPS, verdict=True, r0=True, status=True, regs=True,
                   counters=cnt, generic=generic, mem=mem, **kw)
    # the production launch (verdict only: the liveness-pruned register init)
    v = prog.run(frames, n=n, max_steps=STEPS, generic=generic, **kw)
    torch.cuda.synchronize()
    out = dict(status=res.status.cpu().numpy(), r0=res.r0.cpu().numpy().view(np.uint64),
               verdict=res.verdict.cpu().numpy(), regs=res.regs.cpu().numpy().view(np.uint64),
               counters=cnt.cpu().numpy().view(np.uint64), kernel=got_kernel,
               prod_verdict=v.verdict.cpu().numpy())
    prog.close()
    return out


def _vs_oracle(oracle_mod, img, pkts, got, mem_size=1024, r10=512, tag="", max_steps=STEPS):
    op = oracle_mod.Program(img)
    cnt = np.zeros(8, dtype=np.uint64)
    for i, p in enumerate(pkts):
        st, regs, _m, steps = op.run_full(p, mem_size, r10, max_steps)
        ctx = f"{tag} pkt {i} prog {img.hex()}"
        assert got["status"][i] == st, ctx
        if st == 0:
            assert [int(v) for v in got["regs"][i]] == regs, ctx
            cnt[regs[0] if regs[0] < 5 else 5] += 1
        else:
            cnt[6] += 1
        cnt[7] += steps
    assert list(got["counters"]) == list(cnt), tag


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_stack_window_fuzz(cuda, oracle_mod, seed):
    """Random stack programs over fixed-slot batches: the compiled stack-window kernel ==
    the general interpreter (tier 1) == the oracle, every output; production outputs too."""
    from ebpf_emu import _lib

    rng = random.Random(880 + seed)
    n_run = n_stack = 0
    for it in range(40):
        img = gen_stack_program(rng)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        from ebpf_emu import Program

        p = Program(img)
        k = p.stack_window
        p.close()
        if not k:
            continue
        stride = rng.choice([64, 128])
        pkts = [bytes(rng.getrandbits(8) for _ in range(stride)) for _ in range(rng.choice([64, 100, 130]))]
        frames = _fixed_frames(pkts, stride, cuda)
        # (a constant-address load into the window sends the batch to the general interpreter)
        got = _run(img, frames, len(pkts), cuda, stride=stride)
        # (a constant-address load into the window: the loop kernel's stack variant, whose loads
        # all take the store-forwarding overlay)
        # (store mode: the var kernel's stack statement, test_store_mode.py)
        assert got["kernel"] in (_lib.EBPF_KERNEL_JIT_STACK, _lib.EBPF_KERNEL_JIT_LOOP_STACK,
                                 _lib.EBPF_KERNEL_JIT_VAR_STACK, _lib.EBPF_KERNEL_JIT_VARL_STACK,
                                 _lib.EBPF_KERNEL_GENERAL_T1)
        n_stack += got["kernel"] == _lib.EBPF_KERNEL_JIT_STACK
        ref = _run(img, frames, len(pkts), cuda, generic=True, stride=stride)
        assert ref["kernel"] == _lib.EBPF_KERNEL_GENERAL_T1
        for key in ("status", "r0", "verdict", "regs", "counters", "prod_verdict"):
            assert np.array_equal(got[key], ref[key]), (key, seed, it, img.hex())
        _vs_oracle(oracle_mod, img, pkts, got, tag=f"seed {seed} it {it}")
        n_run += 1
    assert n_run >= 20 and n_stack >= 15, (n_run, n_stack)


@pytest.mark.gpu
def test_stack_window_fallbacks(cuda, oracle_mod):
    """Batches the stack-window kernel must not take -- each on the general interpreter, equal
    to the oracle: the window over packet bytes (r10 = 96 with 128-byte slots), r10 not a multiple
    of 4, an image output, the offsets + lens layout, a constant-address load into the window."""
    import torch

    from ebpf_emu import _lib
    from ebpf_emu.asm import assemble

    rng = random.Random(5)
    src = "ldxdw r3, [r1+8]\nstxdw [r10-16], r3\nstb [r10-3], 0x5a\nldxw r0, [r10-14]\n" \
          "ldxb r4, [r10-3]\nadd r0, r4\nexit"
    img = assemble(src)
    pkts = [bytes(rng.getrandbits(8) for _ in range(128)) for _ in range(70)]
    frames = _fixed_frames(pkts, 128, cuda)
    ok = _run(img, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_JIT_STACK, stride=128)
    _vs_oracle(oracle_mod, img, pkts, ok, tag="eligible")
    # (the window over packet bytes: the loop kernel's stack variant, which loads them at the start)
    got = _run(img, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_JIT_LOOP_STACK, stride=128,
               r10=96)
    _vs_oracle(oracle_mod, img, pkts, got, r10=96, tag="r10 96")
    for kw, r10 in ((dict(r10=510), 510), (dict(mem=True), 512)):
        got = _run(img, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_GENERAL_T1, stride=128, **kw)
        _vs_oracle(oracle_mod, img, pkts, got, r10=r10, tag=str(kw))
    lens = torch.tensor(np.full(len(pkts), 128, dtype=np.int16), device=cuda)
    offs = torch.tensor(np.arange(len(pkts), dtype=np.int32) * 128, device=cuda)
    # (offsets + lens: the var tile loop's stack statement)
    got = _run(img, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_JIT_VARL_STACK, offsets=offs,
               lens=lens)
    _vs_oracle(oracle_mod, img, pkts, got, tag="offsets")
    got = _run(img, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_GENERAL_T1, offsets=offs,
               lens=lens, r10=72)  # (other layouts: the window must lie past byte 64)
    _vs_oracle(oracle_mod, img, pkts, got, r10=72, tag="offsets r10 72")
    alias = assemble("stxdw [r10-8], r2\nldxdw r0, [r1+504]\nexit")  # reads the window at r1+504
    got = _run(alias, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_JIT_LOOP_STACK, stride=128)
    _vs_oracle(oracle_mod, alias, pkts, got, tag="constant alias")
    # register-address loads into the window (r3 = len + 376 = 504: not a load-time constant),
    # wholly and partly inside it: the store-forwarding overlay
    alias2 = assemble("stxdw [r10-8], r2\nmov r3, r2\nadd r3, 376\nldxdw r0, [r3+0]\n"
                      "ldxdw r4, [r3-4]\nadd r0, r4\nldxh r4, [r3-1]\nadd r0, r4\nexit")
    got = _run(alias2, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_JIT_STACK, stride=128)
    _vs_oracle(oracle_mod, alias2, pkts, got, tag="register alias (overlay)")


@pytest.mark.gpu
def test_stack_workload_vs_oracle(cuda, oracle_mod):
    """The 5-tuple with its key spilled to the stack (workloads.FIVE_TUPLE_STACK) on 64 Ki + 37
    fixed-slot frames: the stack-window kernel vs the oracle, and the same verdicts as the plain
    5-tuple."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    n = 65536 + 37
    buf = W.frames_fixed(n, 64, 3)
    frames = torch.from_numpy(buf).to(cuda)
    prog = Program(W.program("5tuple_stack"))
    assert prog.stack_window == 16
    b = prog.make_batch(frames, n=n, stride=64)
    assert prog.batch_kernel(b) == _lib.EBPF_KERNEL_JIT_STACK
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    res = prog.run(frames, n=n, stride=64, r0=True, status=True, counters=cnt)
    torch.cuda.synchronize()
    r0, st, ocnt = oracle_mod.Program(W.program("5tuple_stack")).run_batch(buf, n, stride=64, threads=8)
    assert np.array_equal(res.status.cpu().numpy(), st)
    assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), r0)
    assert np.array_equal(cnt.cpu().numpy().view(np.uint64), ocnt)
    r0b, _, _ = oracle_mod.Program(W.program("5tuple")).run_batch(buf, n, stride=64, threads=8)
    assert np.array_equal(r0, r0b)


# Atomics on the stack window and packet-window stores, directed at the reference's corner cases
# (emu.rs:373-437, oracle/ebpf_oracle.c): 64-bit ADD overflow (ST_ARITH, the debug build), the
# 32-bit form's carry into the high word and the recombination's overflow, fetch, XCHG, CMPXCHG
# (equal and not, 32-bit, without fetch: r0 = 0), src == dst and dst == r0 (the dst write-back,
# Q14), and packet stores of every width read back through constant loads.
ATOMIC_PROGRAMS = [
    "lddw r5, 0x7fffffffffffffc0\nstxdw [r10-8], r5\nmov r6, r2\nlock add [r10-8], r6\n"
    "ldxdw r0, [r10-8]\nexit",
    "lddw r5, 0x7fffffffffffffff\nstxdw [r10-8], r5\nmov r6, 1\nlock add32 [r10-8], r6\n"
    "ldxdw r0, [r10-8]\nexit",
    "lddw r5, 0x7ffffffeffffffff\nstxdw [r10-16], r5\nmov r6, 1\nlock fetch add32 [r10-16], r6\n"
    "ldxdw r0, [r10-16]\nadd r0, r6\nexit",
    "ldxdw r3, [r1+8]\nstxdw [r10-8], r3\nldxdw r4, [r1+16]\nlock fetch or [r10-8], r4\n"
    "lock and [r10-8], r3\nlock fetch xor32 [r10-8], r2\nldxdw r0, [r10-8]\nxor r0, r4\nexit",
    "ldxdw r3, [r1+24]\nstxdw [r10-24], r3\nmov r4, r2\nlock xchg [r10-24], r4\n"
    "ldxdw r0, [r10-24]\nadd r0, r4\nexit",
    "ldxdw r0, [r1+0]\nstxdw [r10-8], r0\nmov r4, r2\nlock cmpxchg [r10-8], r4\n"
    "ldxdw r5, [r10-8]\nadd r0, r5\nexit",
    "mov r0, 7\nldxdw r3, [r1+0]\nstxdw [r10-8], r3\nmov r4, r2\nlock cmpxchg [r10-8], r4\n"
    "ldxdw r5, [r10-8]\nadd r0, r5\nexit",
    "ldxw r0, [r1+4]\nstxdw [r10-8], r0\nmov r4, r2\nlock cmpxchg32 [r10-8], r4\n"
    "ldxdw r5, [r10-8]\nadd r0, r5\nexit",
    "ldxdw r3, [r1+0]\nstxdw [r10-8], r3\nlock cmpxchg [r10-8], r2\nexit",
    "mov r3, r10\nstxdw [r3-8], r2\nlock fetch add [r3-8], r3\nldxdw r0, [r10-8]\nadd r0, r3\nexit",
    "mov r0, r10\nstdw [r10-8], 5\nmov r4, 9\nlock cmpxchg [r0-8], r4\nldxdw r5, [r10-8]\n"
    "mov r0, r5\nexit",
    "ldxw r3, [r1+0]\nldxh r4, [r1+4]\nldxw r5, [r1+6]\nldxh r6, [r1+10]\nstxw [r1+0], r5\n"
    "stxh [r1+4], r6\nstxw [r1+6], r3\nstxh [r1+10], r4\nldxdw r0, [r1+0]\nldxw r7, [r1+8]\n"
    "add r0, r7\nexit",
    "stb [r1+63], 0x5a\nsth [r1+13], 0x1234\nstdw [r1+40], 7\nstxdw [r1+21], r2\n"
    "ldxdw r0, [r1+56]\nldxdw r3, [r1+40]\nadd r0, r3\nldxdw r3, [r1+12]\nadd r0, r3\n"
    "ldxdw r3, [r1+20]\nadd r0, r3\nexit",
]


@pytest.mark.gpu
def test_stack_atomics_and_packet_stores(cuda, oracle_mod):
    """ATOMIC_PROGRAMS on fixed-slot frames: the compiled stack-window kernel == the general
    interpreter == the oracle, every output (faults included), on 64- and 128-byte slots; and the
    MAC-swap workload (workloads.MAC_SWAP_TX) the same way."""
    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    rng = random.Random(17)
    for src in ATOMIC_PROGRAMS + [W.MAC_SWAP_TX]:
        img = assemble(src)
        p = Program(img)
        assert p.stack_window, src
        p.close()
        for stride in (64, 128):
            pkts = [bytes(rng.getrandbits(8) for _ in range(stride)) for _ in range(100)]
            frames = _fixed_frames(pkts, stride, cuda)
            got = _run(img, frames, len(pkts), cuda, kernel=_lib.EBPF_KERNEL_JIT_STACK, stride=stride)
            ref = _run(img, frames, len(pkts), cuda, generic=True, stride=stride)
            for key in ("status", "r0", "verdict", "regs", "counters", "prod_verdict"):
                assert np.array_equal(got[key], ref[key]), (key, stride, src)
            _vs_oracle(oracle_mod, img, pkts, got, tag=f"{stride} {src!r}")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_stack_atomics_fuzz(cuda, oracle_mod, seed):
    """Random stack programs with stack atomics and packet-window stores (gen_stack_program
    pw_atomics): compiled == general interpreter == oracle."""
    from ebpf_emu import Program, _lib

    rng = random.Random(990 + seed)
    n_stack = 0
    for it in range(40):
        img = gen_stack_program(rng, pw_atomics=True)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        p = Program(img)
        k = p.stack_window
        p.close()
        if not k:
            continue
        stride = rng.choice([64, 128])
        pkts = [bytes(rng.getrandbits(8) for _ in range(stride)) for _ in range(rng.choice([64, 100]))]
        frames = _fixed_frames(pkts, stride, cuda)
        got = _run(img, frames, len(pkts), cuda, stride=stride)
        # (a store through an unknown pointer: store mode, the var kernel's stack statement)
        n_stack += got["kernel"] in (_lib.EBPF_KERNEL_JIT_STACK, _lib.EBPF_KERNEL_JIT_VAR_STACK,
                                     _lib.EBPF_KERNEL_JIT_VARL_STACK)
        ref = _run(img, frames, len(pkts), cuda, generic=True, stride=stride)
        for key in ("status", "r0", "verdict", "regs", "counters", "prod_verdict"):
            assert np.array_equal(got[key], ref[key]), (key, seed, it, img.hex())
        _vs_oracle(oracle_mod, img, pkts, got, tag=f"seed {seed} it {it}")
    assert n_stack >= 12, n_stack


# ---------------------------------------------------------------------------------------------
# Memory tier 0.5 on the other layouts (ebpf_tile_jit_var_stack): offsets + lens (a pcap capture),
# stride + lens, and xdp_md batches in place, packets of any length -- short ones (the preloaded
# window's bytes past the packet are zeros) and ones reaching into the stack window (its bytes
# loaded from the packet at the start)
VAR_LAYOUTS = {
    "offsets16": dict(offsets_layout=True, align=16),
    "offsets_mis3": dict(offsets_layout=True, misalign=3),
    "stride_lens": dict(),
    "xdp_offsets": dict(offsets_layout=True, align=16, xdp=True),
    "xdp_stride_lens": dict(xdp=True),
}


def _var_packets(rng, n):
    lens = [0, 1, 5, 13, 14, 34, 60, 63, 64, 65, 100, 200, 470, 490, 500, 505, 511, 600, 1000]
    return [bytes(rng.getrandbits(8) for _ in range(rng.choice(lens))) for _ in range(n)]


def _run_var(img, pkts, dev, layout, generic=False, max_steps=STEPS):
    import torch

    from ebpf_emu import Program
    from test_gpu_parity import _stage

    layout = dict(layout)
    xdp = layout.pop("xdp", False)
    frames, kw = _stage(pkts, dev, **layout)
    prog = Program(img)
    b = prog.make_batch(frames, max_steps=max_steps, generic=generic, xdp_md=xdp, **kw)
    kernel = prog.batch_kernel(b, None, dev.index or 0)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    res = prog.run(frames, max_steps=max_steps, r0=True, status=True, regs=True, counters=cnt,
                   generic=generic, xdp_md=xdp, **kw)
    v = prog.run(frames, max_steps=max_steps, xdp_md=xdp, generic=generic, **kw)  # production
    torch.cuda.synchronize()
    out = dict(status=res.status.cpu().numpy(), r0=res.r0.cpu().numpy().view(np.uint64),
               verdict=res.verdict.cpu().numpy(), regs=res.regs.cpu().numpy().view(np.uint64),
               counters=cnt.cpu().numpy().view(np.uint64), kernel=kernel,
               prod_verdict=v.verdict.cpu().numpy())
    prog.close()
    return out, xdp


def _images_of(pkts, xdp):
    import struct

    return [struct.pack("<II", 8, 8 + len(p)) + p for p in pkts] if xdp else pkts


@pytest.mark.gpu
@pytest.mark.parametrize("layout", sorted(VAR_LAYOUTS))
def test_stack_window_fuzz_var(cuda, oracle_mod, layout):
    """Random stack programs (with and without stack atomics and packet-window stores) on the
    other layouts: the var kernel's stack statement == the general interpreter == the oracle on
    the same images, every output, the production verdicts too."""
    from ebpf_emu import Program, _lib

    rng = random.Random(zlib.crc32(layout.encode()))
    n_stack = 0
    for it in range(30):
        img = gen_stack_program(rng, pw_atomics=it % 2 == 1)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        p = Program(img)
        k = p.stack_window
        p.close()
        if not k:
            continue
        pkts = _var_packets(rng, rng.choice([64, 100, 130]))
        got, xdp = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout])
        assert got["kernel"] in (_lib.EBPF_KERNEL_JIT_VAR_STACK, _lib.EBPF_KERNEL_JIT_VARL_STACK,
                                 _lib.EBPF_KERNEL_JIT_LOOP_STACK, _lib.EBPF_KERNEL_GENERAL_T1)
        n_stack += got["kernel"] in (_lib.EBPF_KERNEL_JIT_VAR_STACK, _lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK)
        ref, _ = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout], generic=True)
        assert ref["kernel"] == _lib.EBPF_KERNEL_GENERAL_T1
        ok = got["status"] != 7  # (ST_BADPKT lanes have no registers: main.rs:20-21 panics)
        for key in ("status", "verdict", "counters", "prod_verdict"):
            assert np.array_equal(got[key], ref[key]), (key, layout, it, img.hex())
        for key in ("r0", "regs"):
            assert np.array_equal(got[key][ok], ref[key][ok]), (key, layout, it, img.hex())
        _vs_oracle(oracle_mod, img, _images_of(pkts, xdp), got, tag=f"{layout} it {it}")
    assert n_stack >= 8, n_stack


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["offsets_mis3", "xdp_offsets"])
def test_stack_workloads_var(cuda, oracle_mod, layout):
    """ATOMIC_PROGRAMS, the key-spilling 5-tuple and the MAC-swap reflector on the other layouts,
    against the oracle and the general interpreter."""
    from ebpf_emu import _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    rng = random.Random(31)
    for src in ATOMIC_PROGRAMS + [W.MAC_SWAP_TX, W.FIVE_TUPLE_STACK]:
        img = assemble(src)
        pkts = _var_packets(rng, 150)
        got, xdp = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout])
        # (offsets + lens: the var tile loop's stack statement; stride + lens the var kernel's)
        assert got["kernel"] in (_lib.EBPF_KERNEL_JIT_VAR_STACK, _lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK), src
        ref, _ = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout], generic=True)
        for key in ("status", "verdict", "counters"):
            assert np.array_equal(got[key], ref[key]), (key, layout, src)
        _vs_oracle(oracle_mod, img, _images_of(pkts, xdp), got, tag=f"{layout} {src!r}")


def test_large_stack_programs_compile():
    """Stack-window programs of 63-256 micro-ops (past the tile interpreter's tables) are memory
    tier 0.5 too: compiled (the compiler-only tables), with the window in registers."""
    from ebpf_emu import Program

    rng = random.Random(4048)
    n_ok = 0
    for it in range(40):
        img = gen_stack_program(rng, n=rng.randrange(70, 200), pw_atomics=it % 2 == 1)
        p = Program(img)
        if p.stack_window:
            assert len(p.instructions) > 62
            assert p.compile(), img.hex()
            assert "; stack window:" in p.jit_asm(1)
            n_ok += 1
        p.close()
    assert n_ok >= 10, n_ok


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed", "offsets_mis3", "xdp_offsets"])
def test_large_stack_programs(cuda, oracle_mod, layout):
    """Stack-window programs of 63-256 micro-ops on the compiled stack kernels == the general
    interpreter == the oracle."""
    from ebpf_emu import Program, _lib

    rng = random.Random(zlib.crc32(b"large" + layout.encode()))
    n_stack = 0
    for it in range(18):
        img = gen_stack_program(rng, n=rng.randrange(70, 200), pw_atomics=it % 2 == 1)
        p = Program(img)
        k = p.stack_window
        p.close()
        if not k:
            continue
        if layout == "fixed":
            pkts = [bytes(rng.getrandbits(8) for _ in range(128)) for _ in range(100)]
            frames = _fixed_frames(pkts, 128, cuda)
            got = _run(img, frames, len(pkts), cuda, stride=128)
            ref = _run(img, frames, len(pkts), cuda, generic=True, stride=128)
            want = _lib.EBPF_KERNEL_JIT_STACK
            xdp = False
        else:
            pkts = _var_packets(rng, 100)
            got, xdp = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout])
            ref, _ = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout], generic=True)
            want = _lib.EBPF_KERNEL_JIT_VAR_STACK
        n_stack += got["kernel"] in (want, _lib.EBPF_KERNEL_JIT_VARL_STACK,
                                     _lib.EBPF_KERNEL_JIT_LOOP_STACK)
        ok = got["status"] != 7
        for key in ("status", "verdict", "counters", "prod_verdict"):
            assert np.array_equal(got[key], ref[key]), (key, layout, it, img.hex())
        for key in ("r0", "regs"):
            assert np.array_equal(got[key][ok], ref[key][ok]), (key, layout, it, img.hex())
        _vs_oracle(oracle_mod, img, _images_of(pkts, xdp), got, tag=f"{layout} it {it}")
    assert n_stack >= 4, n_stack


# ---------------------------------------------------------------------------------------------
# Stack-window programs with loops (or a binding step budget): the loop kernel's stack variant
# (ebpf_tile_jit_loop_stack). STACK_SUM keeps its running sum at r10 - 8 (workloads.CHECKSUM_STACK
# is the checksum written that way).
STACK_SUM = """
    mov r0, 0
    stdw [r10-8], 0
    mov r3, 0
    jge r3, r2, done
loop:
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    ldxdw r6, [r10-8]
    add r6, r5
    stxdw [r10-8], r6
    add r3, 1
    jlt r3, r2, loop
done:
    ldxdw r0, [r10-8]
    exit
"""


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["offsets16", "offsets_mis3", "stride_lens", "xdp_offsets"])
def test_stack_loop_programs(cuda, oracle_mod, layout):
    """Random stack-window loop programs (gen_stack_loop_program) and STACK_SUM: the loop
    kernel's stack variant == the general interpreter == the oracle, every output, budgets that
    bind included; the forward 5-tuple-with-key under a binding budget too."""
    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    rng = random.Random(zlib.crc32(b"loops" + layout.encode()))
    progs = [assemble(STACK_SUM), W.program("checksum_stack"), W.program("5tuple_stack")]
    progs += [gen_stack_loop_program(rng) for _ in range(16)]
    n_stack = 0
    for it, img in enumerate(progs):
        p = Program(img)
        k, prom = p.stack_window, p.promoted
        p.close()
        if not k:
            continue
        for steps in ((3000, 37) if it % 2 == 0 else (3000,)):
            pkts = _var_packets(rng, rng.choice([64, 100]))
            got, xdp = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout], max_steps=steps)
            if it == 2 and steps == 3000:  # (forward, budget that cannot bind: forward kernels)
                assert got["kernel"] in (_lib.EBPF_KERNEL_JIT_VAR_STACK,
                                         _lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK), layout
            else:
                # (the route of the production outputs: a promoted program's own loop kernel,
                # test_promote.py; every output asked for below runs the stack loop kernel)
                want = _lib.EBPF_KERNEL_JIT_LOOP if prom else _lib.EBPF_KERNEL_JIT_LOOP_STACK
                assert got["kernel"] == want, (layout, it, img.hex())
                n_stack += 1
            ref, _ = _run_var(img, pkts, cuda, VAR_LAYOUTS[layout], generic=True, max_steps=steps)
            ok = got["status"] != 7
            for key in ("status", "verdict", "counters", "prod_verdict"):
                assert np.array_equal(got[key], ref[key]), (key, layout, it, steps, img.hex())
            for key in ("r0", "regs"):
                assert np.array_equal(got[key][ok], ref[key][ok]), (key, layout, it, steps, img.hex())
            _vs_oracle(oracle_mod, img, _images_of(pkts, xdp), got, tag=f"{layout} it {it}",
                       max_steps=steps)
    assert n_stack >= 12, n_stack


_FALLBACK_CHILD = r"""
import json, sys, random
import numpy as np, torch
sys.path[:0] = sys.argv[1:3]
from ebpf_emu import Program, _lib
from ebpf_emu import workloads as W
from ebpf_emu.asm import assemble
from fuzzgen import gen_stack_loop_program, gen_stack_program
rng = random.Random(4242)
progs = [assemble(src) for src, k in DIRECTED if k] + [W.program("5tuple_stack"),
         W.program("checksum_stack"), W.program("mac_swap_tx")]
progs += [gen_stack_loop_program(rng) for _ in range(4)] + [gen_stack_program(rng) for _ in range(4)]
dev = torch.device("cuda", 0)
out = []
for img in progs:
    p = Program(img)
    compiled = p.compile()
    pkts = [bytes(rng.getrandbits(8) for _ in range(64)) for _ in range(70)]
    buf = np.frombuffer(b"".join(pkts), dtype=np.uint8)
    frames = torch.tensor(buf, device=dev)
    b = p.make_batch(frames, n=len(pkts), stride=64, max_steps=20000)
    kern = p.batch_kernel(b, _lib.BatchOut(), 0)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    res = p.run(frames, n=len(pkts), stride=64, max_steps=20000, r0=True, status=True, regs=True,
                counters=cnt)
    torch.cuda.synchronize()
    out.append(dict(img=img.hex(), kernel=int(kern), window=p.stack_window, pkts=[x.hex() for x in pkts],
                    status=res.status.cpu().tolist(),
                    regs=res.regs.cpu().numpy().view(np.uint64).tolist(),
                    counters=cnt.cpu().numpy().view(np.uint64).tolist()))
    p.close()
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_stack_compile_failure_falls_back(cuda, oracle_mod):
    """A stack-window program whose compilation fails (EBPFEMU_TEST_FAIL_STACK_JIT=1 forces it)
    runs on the general interpreter's tier 1 -- never on tile_kernel's loop mode, whose tables
    may already be on the device and which has no stores -- with the oracle's results."""
    import json
    import os
    import subprocess
    import sys

    from ebpf_emu import _lib

    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = "DIRECTED = %r\n" % (DIRECTED,) + _FALLBACK_CHILD
    env = dict(os.environ, EBPFEMU_TEST_FAIL_STACK_JIT="1")
    r = subprocess.run([sys.executable, "-c", code, os.path.join(root, "ebpf-emu_amd"), here],
                       capture_output=True, text=True, timeout=150, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(res) >= 20
    for d in res:
        assert d["window"] == 0, d["img"]  # the fallback dropped the stack plan
        assert d["kernel"] == _lib.EBPF_KERNEL_GENERAL_T1, (d["img"], d["kernel"])
        got = dict(status=np.array(d["status"]), regs=np.array(d["regs"], dtype=np.uint64),
                   counters=np.array(d["counters"], dtype=np.uint64))
        _vs_oracle(oracle_mod, bytes.fromhex(d["img"]), [bytes.fromhex(x) for x in d["pkts"]],
                   got, tag="fallback", max_steps=20000)
