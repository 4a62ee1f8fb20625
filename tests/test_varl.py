"""The var tile loop (ebpf_tile_jit_varl): offsets + lens batches -- a capture's
or a NIC ring's layout -- of compiled forward programs, the wave's tiles in one asm statement with
double-buffered windows. Every output against the C oracle (oracle/, restating emu.rs / mmu.rs /
main.rs) and against the general interpreter on the same batch, bit-exact: aligned tiles (LDS-DMA
windows), tiles of unaligned packets (DMA'd straight from the packets, a short packet's last chunk
from the aligned block below and shifted in LDS), partial tiles (handed back to the C++ and
staged lane by lane), packets shorter than the window, lengths absent, init_regs / r0 / status / register outputs, xdp_md in
place, and a wave running more than the 511 tiles of one statement entry."""
import os
import random

import numpy as np
import pytest

from fuzzgen import gen_packet, gen_program
from test_gpu_parity import STEPS, _check_prod_against_oracle

pytestmark = pytest.mark.gpu


def _mixed(pkts, dev, bad_every=0, lens=True, align=None):
    """Offsets layout, every packet 16-byte aligned except each bad_every-th one (at +3): a tile
    holding one is DMA'd straight from its unaligned packets. align(i) -> the packet's address
    mod 16 instead, when given. Returns (frames, kwargs)."""
    import torch

    offs, pos, chunks = [], 0, []
    for i, p in enumerate(pkts):
        want = 3 if bad_every and i % bad_every == bad_every - 1 else 0
        if align is not None:
            want = align(i)
        pad = (want - pos) % 16
        chunks.append(bytes(pad))
        pos += pad
        offs.append(pos)
        chunks.append(p)
        pos += len(p)
    buf = b"".join(chunks) + bytes(16)
    frames = torch.tensor(np.frombuffer(buf, dtype=np.uint8).copy(), device=dev)
    kw = dict(n=len(pkts), offsets=torch.tensor(np.array(offs, dtype=np.uint32).view(np.int32),
                                                 device=dev))
    if lens:
        ln = np.array([len(p) for p in pkts], dtype=np.uint16)
        kw["lens"] = torch.tensor(ln.view(np.int16), device=dev)
    return frames, kw


def _route(prog, frames, kw, **extra):
    return prog.batch_kernel(prog.make_batch(frames, **kw, **extra))


def _outputs(prog, frames, kw, dev, generic=False, regs=False, **extra):
    import torch

    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    v = prog.run(frames, max_steps=STEPS, verdict=True, counters=cnt, generic=generic, **kw,
                 **extra)
    rs = prog.run(frames, max_steps=STEPS, verdict=False, r0=True, status=True, regs=regs,
                  generic=generic, **kw, **extra)
    torch.cuda.synchronize()
    out = dict(verdict=v.verdict.cpu().numpy(), counters=cnt.cpu().numpy().view(np.uint64),
               r0=rs.r0.cpu().numpy().view(np.uint64), status=rs.status.cpu().numpy())
    if regs:
        out["regs"] = rs.regs.cpu().numpy().view(np.uint64)
    return out


def _same(a, b, ctx):
    for k in a:
        assert np.array_equal(a[k], b[k]), f"{ctx}: {k} differs"


def _eq_sensitive(got, want, ctx):
    """got == want, and the comparison is live: the same check fails once one bit of the
    expected array is flipped."""
    got, want = np.asarray(got), np.asarray(want)
    assert np.array_equal(got, want), ctx
    if want.size:
        w2 = want.copy()
        w2.reshape(-1).view(np.uint8)[0] ^= 1
        assert not np.array_equal(got, w2), f"{ctx}: a flipped bit went unnoticed"


def _vs_oracle_batch(oracle_mod, img, buf, n, got, ctx, **kw):
    """Every production output of `got` (verdict, r0 where the packet completed, status,
    counters) against the C oracle's run_batch of the same packets (oracle/ebpf_oracle.c, which
    restates emu.rs / mmu.rs / main.rs)."""
    r0, st, cnt = oracle_mod.Program(img).run_batch(buf, n, threads=8, max_steps=STEPS, **kw)
    _eq_sensitive(got["status"], st, f"{ctx}: status")
    ok = st == 0
    _eq_sensitive(got["r0"][ok], r0[ok], f"{ctx}: r0")
    want_v = np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8)
    _eq_sensitive(got["verdict"], want_v, f"{ctx}: verdict")
    _eq_sensitive(got["counters"], cnt, f"{ctx}: counters")


@pytest.mark.parametrize("seed", range(4))
def test_varl_fuzz(cuda, oracle_mod, seed):
    """Random forward programs over random packets (0..80 bytes) in offsets + lens batches of
    64..300 packets: aligned, every tile staged, and mixed; the route is the var tile loop; every
    output == the oracle's and == the general interpreter's, registers included."""
    from ebpf_emu import Program, _lib

    rng = random.Random(7100 + seed)
    done = 0
    for it in range(30):
        img = gen_program(rng, allow_loops=False, tier0=True)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        prog = Program(img)
        if not prog.forward_only:
            prog.close()
            continue
        pkts = [gen_packet(rng) for _ in range(rng.choice([64, 65, 100, 130, 300]))]
        bad = rng.choice([0, 0, 1, 37])
        frames, kw = _mixed(pkts, cuda, bad_every=bad)
        k = _route(prog, frames, kw, max_steps=STEPS)
        if k != _lib.EBPF_KERNEL_JIT_VARL:  # (a program the compiler does not take)
            prog.close()
            continue
        got = _outputs(prog, frames, kw, cuda, regs=True)
        ref = _outputs(prog, frames, kw, cuda, generic=True, regs=True)
        ctx = f"seed {seed} it {it} bad {bad} prog {img.hex()}"
        _same(got, ref, ctx)
        _check_prod_against_oracle(oracle_mod, img, pkts, got, tag=ctx)
        prog.close()
        done += 1
    assert done >= 15


@pytest.mark.parametrize("seed", range(3))
def test_varl_any_alignment(cuda, oracle_mod, seed):
    """Every packet at a random address mod 16 (0..15) and 0..80 bytes long, so most tiles are
    DMA'd from unaligned packets and short packets' last chunks take the aligned-block path and
    the shift at the tile's top (gen_tile.py tailfix): random forward programs and the bench
    programs, every output == the oracle's and == the general interpreter's, registers included;
    one capture-like batch (records at 8 mod 16) of the 5-tuple too."""
    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    rng = random.Random(7300 + seed)
    imgs = [W.program(n) for n in ("5tuple", "acl", "mac_swap_tx", "5tuple_xdp", "nat")]
    while len(imgs) < 16:
        img = gen_program(rng, allow_loops=False, tier0=True)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        imgs.append(img)
    done = 0
    for it, img in enumerate(imgs):
        prog = Program(img)
        if not prog.forward_only:
            prog.close()
            continue
        n = rng.choice([64, 128, 200, 640])
        pkts = [(gen_packet(rng) + bytes(rng.getrandbits(8) for _ in range(80)))[
            :rng.choice([0, 1, 7, 15, 16, 17, 33, 47, 48, 49, 63, 64, 65, 80])] for _ in range(n)]
        fixed_m = rng.choice([None, 8, 4, 1])
        frames, kw = _mixed(pkts, cuda, align=(lambda i: fixed_m) if fixed_m is not None
                            else (lambda i: rng.randrange(16)))
        k = _route(prog, frames, kw, max_steps=STEPS)
        if k not in (_lib.EBPF_KERNEL_JIT_VARL, _lib.EBPF_KERNEL_JIT_VARL_STACK):
            prog.close()
            continue
        regs = k == _lib.EBPF_KERNEL_JIT_VARL  # (store mode: the production outputs)
        got = _outputs(prog, frames, kw, cuda, regs=regs)
        ref = _outputs(prog, frames, kw, cuda, generic=True, regs=regs)
        ctx = f"seed {seed} it {it} m {fixed_m} kernel {k} prog {img.hex()}"
        _same(got, ref, ctx)
        _check_prod_against_oracle(oracle_mod, img, pkts, got, tag=ctx)
        prog.close()
        done += 1
    assert done >= 8


@pytest.mark.parametrize("name", ["5tuple", "drop", "acl", "5tuple_stack", "mac_swap_tx"])
def test_varl_workloads_vs_fixed(cuda, oracle_mod, name):
    """The bench programs (the stack-window ones on the stack statement) over 200 013 of the
    workload's frames as an offsets + lens batch
    (80-byte slots, every 5th packet misaligned in a quarter of the tiles) and with lengths
    absent: verdicts, r0, status and counters == the C oracle's on the same frames, and == the
    compiled fixed-slot kernel's."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    n = 200_000 + 13  # (a partial last tile)
    prog = Program(W.program(name))
    buf = W.frames_fixed(n, 64, 3)
    fr = torch.from_numpy(buf).to(cuda)
    ref = _outputs(prog, fr, dict(n=n, stride=64), cuda)
    _vs_oracle_batch(oracle_mod, W.program(name), buf, n, ref, f"{name} fixed", stride=64)
    stack = name in ("5tuple_stack", "mac_swap_tx")  # (memory tier 0.5: the stack statements)
    assert _route(prog, fr, dict(n=n, stride=64)) == (
        _lib.EBPF_KERNEL_JIT_STACK if stack else _lib.EBPF_KERNEL_JIT_FIXED_OCC)  # (test_occ.py)
    # the same frames at offsets: slots of 80 bytes, packet i at 80 i (+3 for some)
    slot = 80
    big = np.zeros((n, slot), dtype=np.uint8)
    shift = np.zeros(n, dtype=np.int64)
    tiles = np.arange(n) // 64
    shift[(tiles % 4 == 1) & (np.arange(n) % 5 == 0)] = 3
    for s in (0, 3):
        m = shift == s
        big[m, s:s + 64] = buf.reshape(n, 64)[m]
    offs = (np.arange(n, dtype=np.int64) * slot + shift).astype(np.uint32)
    frames = torch.from_numpy(big.reshape(-1)).to(cuda)
    o = torch.from_numpy(offs.view(np.int32)).to(cuda)
    ln = torch.from_numpy(np.full(n, 64, dtype=np.int16)).to(cuda)
    for kw in (dict(n=n, offsets=o, lens=ln), dict(n=n, offsets=o, stride=64)):
        assert _route(prog, frames, kw) == (_lib.EBPF_KERNEL_JIT_VARL_STACK if stack
                                            else _lib.EBPF_KERNEL_JIT_VARL)
        got = _outputs(prog, frames, kw, cuda)
        _vs_oracle_batch(oracle_mod, W.program(name), big.reshape(-1), n, got,
                         f"{name} {sorted(kw)}", offsets=offs,
                         lens=np.full(n, 64, dtype=np.uint16) if "lens" in kw else None,
                         stride=0 if "lens" in kw else 64)
        _same(got, ref, f"{name} {sorted(kw)}")
    prog.close()


def test_varl_statement_reentry(cuda, oracle_mod):
    """One workgroup (EBPFEMU_VARL_WGS=1: 4 waves) over 3000 tiles: each wave runs 750 tiles, so
    the statement returns after 511 and comes back (the packed counter buckets are unpacked in
    between); misaligned tiles on both sides of the return. Against the C oracle and the
    fixed-slot kernel."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    n = 3000 * 64 - 7
    prog = Program(W.program("5tuple"))
    buf = W.frames_fixed(n, 64, 5)
    fr = torch.from_numpy(buf).to(cuda)
    ref = _outputs(prog, fr, dict(n=n, stride=64), cuda)
    pkts_shift = np.zeros(n, dtype=np.int64)
    pkts_shift[np.isin(np.arange(n) // 64, [3, 510, 511, 512, 2043, 2044, 2045, 2999])] = 1
    slot = 80
    big = np.zeros((n, slot), dtype=np.uint8)
    for s in (0, 1):
        m = pkts_shift == s
        big[m, s:s + 64] = buf.reshape(n, 64)[m]
    offs = (np.arange(n, dtype=np.int64) * slot + pkts_shift).astype(np.uint32)
    frames = torch.from_numpy(big.reshape(-1)).to(cuda)
    kw = dict(n=n, offsets=torch.from_numpy(offs.view(np.int32)).to(cuda),
              lens=torch.from_numpy(np.full(n, 64, dtype=np.int16)).to(cuda))
    os.environ["EBPFEMU_VARL_WGS"] = "1"
    try:
        assert _route(prog, frames, kw) == _lib.EBPF_KERNEL_JIT_VARL
        got = _outputs(prog, frames, kw, cuda)
    finally:
        del os.environ["EBPFEMU_VARL_WGS"]
    _vs_oracle_batch(oracle_mod, W.program("5tuple"), big.reshape(-1), n, got, "reentry",
                     offsets=offs, lens=np.full(n, 64, dtype=np.uint16))
    _same(got, ref, "reentry")
    prog.close()


def test_varl_layout_routes(cuda, oracle_mod):
    """Which batches take the var tile loop: offsets with lengths (4-byte aligned) or without;
    not a length array at a 2-byte offset, not final images (the var kernel) -- same outputs
    either way, against the oracle."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    rng = random.Random(5)
    pkts = [gen_packet(rng, 120) for _ in range(333)]
    img = W.program("5tuple")
    prog = Program(img)
    frames, kw = _mixed(pkts, cuda, bad_every=0)
    assert _route(prog, frames, kw) == _lib.EBPF_KERNEL_JIT_VARL
    got = _outputs(prog, frames, kw, cuda)
    _check_prod_against_oracle(oracle_mod, img, pkts, got, tag="aligned lens")
    # lengths at a 2-byte aligned address: the var kernel
    ln2 = torch.zeros(len(pkts) + 1, dtype=torch.int16, device=cuda)
    ln2[1:] = kw["lens"]
    kw2 = dict(kw, lens=ln2[1:])
    assert kw2["lens"].data_ptr() % 4 == 2
    assert _route(prog, frames, kw2) == _lib.EBPF_KERNEL_JIT_VAR
    _same(_outputs(prog, frames, kw2, cuda), got, "lens at +2")
    # final images (the var kernel): the same r0
    res = prog.run(frames, mem=True, r0=True, status=True, max_steps=STEPS, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), got["r0"])
    # no lengths: every packet `stride` bytes long (here 64)
    pk64 = [p[:64].ljust(64, b"\0") for p in pkts]
    frames, kw = _mixed(pk64, cuda, bad_every=7, lens=False)
    kw["stride"] = 64
    assert _route(prog, frames, kw) == _lib.EBPF_KERNEL_JIT_VARL
    _check_prod_against_oracle(oracle_mod, img, pk64, _outputs(prog, frames, kw, cuda),
                               tag="no lens")
    prog.close()


def test_varl_xdp_md(cuda, oracle_mod):
    """xdp_md batches in place on the var tile loop (the ctx synthesised in the preloaded window,
    BASE = packet - 8, LEN = 8 + len): every output, registers included, == the C oracle's on the
    ctx-prefixed images [u32 8][u32 8 + len][packet] (xdp.rs:16-20 handed to main.rs), and == the
    general interpreter's in-place images."""
    import struct

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    rng = random.Random(11)
    pkts = [gen_packet(rng, 100) for _ in range(260)]
    img = W.program("5tuple_xdp")
    prog = Program(img)
    op = oracle_mod.Program(img)
    images = [struct.pack("<II", 8, 8 + len(p)) + p for p in pkts]
    for bad in (0, 9):
        frames, kw = _mixed(pkts, cuda, bad_every=bad)
        kw["xdp_md"] = True
        assert _route(prog, frames, kw) == _lib.EBPF_KERNEL_JIT_VARL
        got = _outputs(prog, frames, kw, cuda, regs=True)
        ref = _outputs(prog, frames, kw, cuda, generic=True, regs=True)
        want = dict(status=[], r0=[], regs=[], counters=np.zeros(8, dtype=np.uint64))
        for im in images:
            st, oregs, _, steps = op.run_full(im, 1024, 512, STEPS)
            want["status"].append(st)
            want["regs"].append(oregs if st == 0 else [0] * 11)
            want["counters"][(oregs[0] if oregs[0] < 5 else 5) if st == 0 else 6] += 1
            want["counters"][7] += steps
        st = np.array(want["status"], dtype=np.uint8)
        ok = st == 0
        oregs = np.array(want["regs"], dtype=np.uint64)
        _eq_sensitive(got["status"], st, f"xdp bad {bad}: status")
        _eq_sensitive(got["regs"][ok], oregs[ok], f"xdp bad {bad}: regs")
        _eq_sensitive(got["r0"][ok], oregs[ok, 0], f"xdp bad {bad}: r0")
        _eq_sensitive(got["counters"], want["counters"], f"xdp bad {bad}: counters")
        _same(got, ref, f"xdp bad {bad}")
    prog.close()


@pytest.mark.parametrize("name", ["5tuple", "5tuple_stack", "nat"])
def test_varl_stride_lens(cuda, oracle_mod, name):
    """Stride + lens batches (16-byte aligned slots of 80 bytes, packets 0..80 bytes long) on the
    var tile loop's stride mode (no offsets: addresses from the slot index): == the oracle and the
    general interpreter; the NAT rewrite in store mode with lanes that deoptimize (ports past the
    window) and their deopt pass."""
    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from test_store_mode import _nat_packets

    rng = random.Random(404)
    img = W.program(name)
    pkts = (_nat_packets(rng, 700) if name == "nat" else [gen_packet(rng) for _ in range(700)])
    pkts = [p[:80] for p in pkts]
    prog = Program(img)
    import torch

    buf = np.zeros((len(pkts), 80), dtype=np.uint8)
    for i, p in enumerate(pkts):
        buf[i, :len(p)] = np.frombuffer(p, dtype=np.uint8)
    frames = torch.from_numpy(buf.reshape(-1)).to(cuda)
    ln = np.array([len(p) for p in pkts], dtype=np.uint16)
    kw = dict(n=len(pkts), stride=80, lens=torch.from_numpy(ln.view(np.int16)).to(cuda))
    stack = name != "5tuple"
    assert _route(prog, frames, kw) == (_lib.EBPF_KERNEL_JIT_VARL_STACK if stack
                                        else _lib.EBPF_KERNEL_JIT_VARL)
    got = _outputs(prog, frames, kw, cuda, regs=True)
    ref = _outputs(prog, frames, kw, cuda, generic=True, regs=True)
    ok = got["status"] != 7  # (ST_BADPKT lanes: no registers, main.rs:20-21 panics)
    for k in ("verdict", "counters", "status"):
        assert np.array_equal(got[k], ref[k]), (name, k)
    for k in ("r0", "regs"):
        assert np.array_equal(got[k][ok], ref[k][ok]), (name, k)
    _check_prod_against_oracle(oracle_mod, img, pkts, got, tag=name)
    prog.close()


def test_varl_init_regs(cuda, oracle_mod):
    """Caller-set registers (Emu.state.regs, emu.rs:14-17: batch.init_regs) on the var tile loop
    (the statement's out-of-line initialisation): every output == the C oracle's run with the
    same registers (oracle run_full init_regs), and == the general interpreter's, for random
    forward programs and register sets."""
    import torch

    from ebpf_emu import Program, _lib

    rng = random.Random(77)
    done = 0
    for it in range(12):
        img = gen_program(rng, allow_loops=False, tier0=True)
        prog = Program(img)
        if not prog.forward_only:
            prog.close()
            continue
        pkts = [gen_packet(rng) for _ in range(130)]
        frames, kw = _mixed(pkts, cuda, bad_every=rng.choice([0, 29]))
        regs = [rng.choice([0, 1, 7, 64, 1 << 33, (1 << 64) - 5, rng.getrandbits(64)])
                for _ in range(11)]
        regs[10] = 512
        ir = torch.tensor(np.array(regs, dtype=np.uint64).view(np.int64), device=cuda)
        if _route(prog, frames, kw, init_regs=ir, max_steps=STEPS) != _lib.EBPF_KERNEL_JIT_VARL:
            prog.close()
            continue
        got = _outputs(prog, frames, kw, cuda, regs=True, init_regs=ir)
        ref = _outputs(prog, frames, kw, cuda, generic=True, regs=True, init_regs=ir)
        op = oracle_mod.Program(img)
        ost, oregs = [], []
        for p in pkts:
            st, rr, _, _ = op.run_full(p, 1024, 512, STEPS, init_regs=regs)
            ost.append(st)
            oregs.append(rr if st == 0 else [0] * 11)
        ost = np.array(ost, dtype=np.uint8)
        ok = ost == 0
        oregs = np.array(oregs, dtype=np.uint64)
        _eq_sensitive(got["status"], ost, f"init_regs it {it}: status")
        _eq_sensitive(got["regs"][ok], oregs[ok], f"init_regs it {it}: regs")
        _same(got, ref, f"init_regs it {it} prog {img.hex()}")
        prog.close()
        done += 1
    assert done >= 5
