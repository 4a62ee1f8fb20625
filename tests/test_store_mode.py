"""Store mode: register-address stores into the packet on the compiled kernel (host.cpp
analyze_stack StackPlan::any_dyn, jit.cpp body_store / lds_store_dyn; reference emu.rs:354-372,
mmu.rs:23-30).

A store through a register whose value the load-time dataflow cannot resolve -- a TTL, port or
checksum rewrite behind the variable-length IPv4 header -- used to send the whole program to the
general interpreter's tier 1 (per-packet images in scratch). In store mode the program runs on the
var kernel's stack statement with the lane's 64-byte header window in LDS as the image's bytes
[0, 64): every packet load and store goes through it. A lane whose store leaves the window (or
whose load straddles its end) deoptimizes: the compiled kernel lists its packet, and the general
interpreter re-runs that packet from the start after the launch (the deopt pass), writing its
outputs and counters. Programs are pure functions of the packet image, so the results are the
reference's either way.

CPU: which programs are store mode, and every one of them compiles and assembles.
GPU: compiled == general interpreter == oracle, every output (status, r0, registers, verdicts,
counters, production verdicts), over random store programs on fixed slots, offsets + lens with
short packets, stride + lens and xdp_md batches -- with lanes that deoptimize, fault, or store
past the packet's length -- and the NAT rewrite workload (workloads.NAT_REWRITE) with packets whose
IPv4 options push the port past the window.
"""
import random
import struct
import zlib

import numpy as np
import pytest

from fuzzgen import gen_store_program

STEPS = 20000


def test_store_mode_programs_compile(product_lib):
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    p = Program(W.program("nat"))
    assert p.tier == 1 and p.stack_window == 4 and p.compile() and p.store_mode
    p.close()
    rng = random.Random(77)
    n = 0
    for _ in range(120):
        img = gen_store_program(rng)
        try:
            p = Program(img)
        except Exception:
            continue
        if p.stack_window:
            assert p.compile(), img.hex()
            n += 1
        p.close()
    assert n >= 80, n


def _nat_packets(rng, n, long_options=0.2):
    """Ethernet/IPv4/TCP-UDP frames: TTL 0..255, IHL 5..15 (IHL >= 13 puts the port past the
    64-byte window: those lanes deoptimize), ports 53 / 80 / random, lengths 34..200."""
    out = []
    for _ in range(n):
        ihl = rng.choice([5, 5, 5, 6]) if rng.random() > long_options else rng.randrange(7, 16)
        plen = max(34, 14 + 4 * ihl + rng.choice([0, 2, 4, 8, 20])) + rng.randrange(0, 60)
        b = bytearray(rng.getrandbits(8) for _ in range(plen))
        b[12:14] = b"\x08\x00" if rng.random() < 0.9 else b"\x86\xdd"
        b[14] = 0x40 | ihl
        b[22] = rng.choice([0, 1, 2, 64, 255])
        b[23] = rng.choice([6, 17, 1])
        l4 = 14 + 4 * ihl
        if l4 + 4 <= plen:
            b[l4 + 2:l4 + 4] = struct.pack(">H", rng.choice([53, 80, 80, 443, rng.randrange(65536)]))
        out.append(bytes(b))
    return out


def _check(oracle_mod, img, pkts, got, ref, xdp, tag):
    from test_stack_tier import _images_of, _vs_oracle

    ok = got["status"] != 7  # (ST_BADPKT lanes have no registers: main.rs:20-21 panics)
    for key in ("status", "verdict", "counters", "prod_verdict"):
        assert np.array_equal(got[key], ref[key]), (key, tag, img.hex())
    for key in ("r0", "regs"):
        assert np.array_equal(got[key][ok], ref[key][ok]), (key, tag, img.hex())
    _vs_oracle(oracle_mod, img, _images_of(pkts, xdp), got, tag=tag)


def _assert_no_deopt(ws, prog):
    """No lane left for the general interpreter: the list's count (workspace +0) is 0, and the
    deopt pass either re-ran nothing (+8 == 0) or, for a program proven deopt-free
    (jit.cpp store_mode_no_deopt), was not launched (+8 keeps the test's 0xFFFFFFFF)."""
    w = ws[:12].cpu().numpy().view(np.uint32)
    assert w[0] == 0, ("lanes deoptimized", w)
    assert w[2] == (0xFFFFFFFF if prog.store_mode_no_deopt else 0), w


LAYOUTS = ["fixed64", "fixed128", "offsets16", "offsets_mis3", "stride_lens", "xdp_offsets"]


def _run_layout(img, pkts, dev, layout, generic=False):
    from test_stack_tier import VAR_LAYOUTS, _fixed_frames, _run, _run_var

    if layout.startswith("fixed"):
        stride = int(layout[5:])
        pk = [p[:stride].ljust(stride, b"\0") for p in pkts]
        frames = _fixed_frames(pk, stride, dev)
        return _run(img, frames, len(pk), dev, generic=generic, stride=stride), False, pk
    out, xdp = _run_var(img, pkts, dev, VAR_LAYOUTS[layout], generic=generic)
    return out, xdp, pkts


@pytest.mark.gpu
@pytest.mark.parametrize("layout", LAYOUTS)
def test_store_mode_fuzz(cuda, oracle_mod, layout):
    """Random store-mode programs: the compiled var kernel (+ its deopt pass) == the general
    interpreter == the oracle on every output; the route asserted."""
    from ebpf_emu import Program, _lib
    from test_stack_tier import _var_packets

    rng = random.Random(zlib.crc32(b"store" + layout.encode()))
    n_run = n_sm = 0
    for it in range(28):
        img = gen_store_program(rng)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        p = Program(img)
        k, sm = p.stack_window, p.store_mode
        p.close()
        if not k:
            continue
        pkts = _var_packets(rng, rng.choice([64, 100, 130]))
        got, xdp, pk = _run_layout(img, pkts, cuda, layout)
        # (a program whose only unknown pointer is loaded through is an ordinary stack program)
        if sm:
            # (the var tile loop's stack statement where the layout allows, else the var kernel's)
            assert got["kernel"] in (_lib.EBPF_KERNEL_JIT_VAR_STACK,
                                     _lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK), (layout, img.hex())
            n_sm += 1
        else:
            assert got["kernel"] in (_lib.EBPF_KERNEL_JIT_STACK, _lib.EBPF_KERNEL_JIT_VAR_STACK,
                                     _lib.EBPF_KERNEL_JIT_VARL_STACK,
                                     _lib.EBPF_KERNEL_GENERAL_T1), (layout, img.hex())
        ref, _, _ = _run_layout(img, pkts, cuda, layout, generic=True)
        assert ref["kernel"] == _lib.EBPF_KERNEL_GENERAL_T1
        _check(oracle_mod, img, pk, got, ref, xdp, f"{layout} it {it}")
        n_run += 1
    assert n_run >= 15 and n_sm >= 10, (n_run, n_sm)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed128", "offsets_mis3", "xdp_offsets"])
def test_nat_rewrite_vs_oracle(cuda, oracle_mod, layout):
    """The NAT rewrite workload over frames with IPv4 options (ports past the window: deopt),
    TTLs that drop, short and long frames: compiled == general interpreter == oracle."""
    from ebpf_emu import _lib
    from ebpf_emu import workloads as W

    img = W.program("nat")
    rng = random.Random(5150 + len(layout))
    pkts = _nat_packets(rng, 3000)
    got, xdp, pk = _run_layout(img, pkts, cuda, layout)
    assert got["kernel"] in (_lib.EBPF_KERNEL_JIT_VAR_STACK, _lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK)
    ref, _, _ = _run_layout(img, pkts, cuda, layout, generic=True)
    _check(oracle_mod, img, pk, got, ref, xdp, f"nat {layout}")
    # the workload exercised every path: TX (redirected), PASS, DROP (under xdp_md the program,
    # not written for the ctx convention, reads the ctx-prefixed image: parity only)
    v = got["verdict"]
    if not xdp:
        assert (v == 3).sum() > 50 and (v == 2).sum() > 50 and (v == 1).sum() > 50


@pytest.mark.gpu
def test_nat_workload_full_size(cuda, oracle_mod):
    """The bench's NAT batch (the 5-tuple frames, 1 Mi x 64 B fixed slots, chunk 0 of the pinned
    pool) against the oracle: verdict counters and retired instructions, then the same batch with
    every 16th frame's IHL set to 15 (the port past the window: 1/16 of the lanes deoptimize)."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W
    from ebpf_emu import dist as D

    img = W.program("nat")
    n = 1 << 20
    for deopt in (False, True):
        buf = D.chunk_frames(0, n).copy()
        if deopt:
            v = buf.reshape(n, 64)
            v[::16, 14] = (v[::16, 14] & 0xF0) | 0x0F
        prog = Program(img)
        cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
        res = prog.run(torch.from_numpy(buf).to(cuda), n=n, stride=64, counters=cnt)
        torch.cuda.synchronize()
        r0, st, ocnt = oracle_mod.Program(img).run_batch(buf, n, stride=64, threads=8)
        verdict = np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8)
        assert np.array_equal(res.verdict.cpu().numpy(), verdict), deopt
        assert list(cnt.cpu().numpy().view(np.uint64)) == list(ocnt), deopt
        prog.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed128", "offsets_mis3", "xdp_offsets"])
def test_nat_long_options_no_deopt(cuda, oracle_mod, layout):
    """IPv4 options up to IHL 15 put the NAT's port store at image bytes 74..77, past the 64-byte
    header window: on the var tile loop those stores (and the port loads after them) go to the
    packet's overflow image (jit.cpp ovf_fill, image bytes [64, 128)) instead of deoptimizing --
    the deopt pass re-runs no packet (the workspace word at +8, LaunchArgs::deopt[2]), and every
    output == the general interpreter's == the oracle's."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from test_stack_tier import VAR_LAYOUTS, _fixed_frames

    img = W.program("nat")
    rng = random.Random(77 + len(layout))
    pkts = _nat_packets(rng, 2000, long_options=1.0)
    assert sum(14 + 4 * (p[14] & 15) + 4 > 64 for p in pkts) > 500
    prog = Program(img)
    if layout.startswith("fixed"):
        stride = int(layout[5:])
        pk = [p[:stride].ljust(stride, b"\0") for p in pkts]
        frames = _fixed_frames(pk, stride, cuda)
        kw = dict(n=len(pk), stride=stride)
        xdp = False
    else:
        from test_gpu_parity import _stage

        spec = dict(VAR_LAYOUTS[layout])
        xdp = spec.pop("xdp", False)
        pk = pkts
        frames, kw = _stage(pkts, cuda, **spec)
    b = prog.make_batch(frames, xdp_md=xdp, **kw)
    ws = torch.full((prog.workspace_bytes(b, 0),), 0x55, dtype=torch.uint8, device=cuda)
    ws[:512 + 64 * 8 * 8] = 0  # (launch.h: the deopt words and counter shards start zeroed)
    b = prog.make_batch(frames, xdp_md=xdp, workspace=ws, **kw)
    assert prog.batch_kernel(b) in (_lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK)
    out = _lib.BatchOut()
    r0 = torch.empty(len(pk), dtype=torch.int64, device=cuda)
    st = torch.empty(len(pk), dtype=torch.uint8, device=cuda)
    ws[8:12] = 0xFF
    out.r0, out.status = r0.data_ptr(), st.data_ptr()
    prog.launch(b, out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    _assert_no_deopt(ws, prog)
    gen = prog.run(frames, r0=True, status=True, generic=True, xdp_md=xdp, **kw)
    torch.cuda.synchronize()
    assert torch.equal(st, gen.status)
    ok = st == 0
    assert torch.equal(r0[ok], gen.r0[ok])
    from test_stack_tier import _images_of

    op = oracle_mod.Program(img)
    stn, r0n = st.cpu().numpy(), r0.cpu().numpy().view(np.uint64)
    for i, im in enumerate(_images_of(pk, xdp)):
        s, o0, _ = op.run_packet(im, 1024, 512, 1 << 22)
        assert stn[i] == s, (layout, i)
        if s == 0:
            assert int(r0n[i]) == o0, (layout, i)
    prog.close()


# a packet byte picks where the program stores (r1 + 2 * byte: 0..510, through a register): in
# the header window, in the overflow image, or -- with the batch's r10 at 128 -- past the stack
# window's start (r10 - k): those deoptimize (about three lanes in four)
DEOPT_PROG = """
    ldxb r3, [r1+14]
    lsh r3, 1
    mov r4, r1
    add r4, r3
    stb [r4+0], 0x5a
    ldxb r0, [r4+0]
    ldxb r5, [r1+20]
    add r0, r5
    and r0, 3
    exit
"""


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed128", "offsets_mis3", "big"])
def test_deopt_list_rerun(cuda, oracle_mod, layout):
    """A store-mode batch where most lanes deoptimize (r10 = 128: a store ending past the stack
    window's start r10 - k, which the compiled kernel holds in registers): the var tile loop lists
    them, the deopt pass re-runs them on the general interpreter (host.cpp,
    LaunchArgs::deopt_pass). 128-byte slots, unaligned offsets + lens and 300 000 packets; two
    launches on one workspace (the pass resets the list's words for the next); status, r0 and
    counters == the general interpreter's == the oracle's, and the re-run count (workspace +8) ==
    the lanes whose store ends past r10 - k."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu.asm import assemble
    from test_stack_tier import VAR_LAYOUTS, _fixed_frames

    img = assemble(DEOPT_PROG)
    rng = random.Random(404 + len(layout))
    n = 300_000 if layout == "big" else 3000
    pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 10, 15, 21, 60, 64, 100, 128])))
            for _ in range(n)]
    prog = Program(img)
    if layout != "offsets_mis3":
        stride = 128
        pk = [p[:stride].ljust(stride, b"\0") for p in pkts]
        frames = _fixed_frames(pk, stride, cuda)
        kw = dict(n=len(pk), stride=stride)
    else:
        from test_gpu_parity import _stage

        pk = pkts
        frames, kw = _stage(pkts, cuda, **VAR_LAYOUTS[layout])
    b = prog.make_batch(frames, r10=128, **kw)
    assert prog.batch_kernel(b) in (_lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK)
    ws = torch.zeros(prog.workspace_bytes(b, 0), dtype=torch.uint8, device=cuda)
    b = prog.make_batch(frames, r10=128, workspace=ws, **kw)
    gcnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    gen = prog.run(frames, r0=True, status=True, generic=True, counters=gcnt, r10=128, **kw)
    op = oracle_mod.Program(img)
    s0 = 128 - prog.stack_window
    want_rerun = sum(1 for p in pk if len(p) > 14 and 2 * p[14] + 1 > s0)
    assert want_rerun > n // 2
    for rep in range(2):
        out = _lib.BatchOut()
        r0 = torch.empty(len(pk), dtype=torch.int64, device=cuda)
        st = torch.empty(len(pk), dtype=torch.uint8, device=cuda)
        cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
        out.r0, out.status, out.counters = r0.data_ptr(), st.data_ptr(), cnt.data_ptr()
        prog.launch(b, out, torch.cuda.current_stream())
        torch.cuda.synchronize()
        words = ws[:16].cpu().numpy().view(np.uint32)
        # the list's count and done words (launch.h kWsDeoptOff) reset for the next launch
        assert words[0] == 0 and words[1] == 0, (rep, words)
        assert words[2] == want_rerun, (rep, words[2], want_rerun)
        assert torch.equal(st, gen.status), rep
        ok = st == 0
        assert torch.equal(r0[ok], gen.r0[ok]), rep
        assert torch.equal(cnt, gcnt), (rep, cnt, gcnt)
        stn, r0n = st.cpu().numpy(), r0.cpu().numpy().view(np.uint64)
        for i in range(0, len(pk), 1 if n <= 3000 else 97):
            s, o0, _ = op.run_packet(pk[i], 1024, 128, 1 << 22)
            assert stn[i] == s, (layout, i)
            if s == 0:
                assert int(r0n[i]) == o0, (layout, i)
    prog.close()


# a pointer to image byte 57..64 (a packet byte picks it); a store just below it into the window,
# on every other packet a store past byte 64 (the overflow image: the lane is dirty), then 8-, 4-
# and 2-byte loads through it that straddle the window's end
STRADDLE_PROG = """
    ldxb r3, [r1+14]
    and r3, 7
    mov r4, r1
    add r4, r3
    add r4, 57
    stb [r4-1], 0x33
    ldxb r5, [r1+15]
    and r5, 1
    jeq r5, 0, nost
    stb [r4+8], 0x77
nost:
    ldxdw r0, [r4+0]
    ldxw r6, [r4+0]
    ldxh r7, [r4+1]
    xor r0, r6
    xor r0, r7
    exit
"""


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed128", "offsets_mis3", "xdp_offsets"])
def test_straddling_loads_no_deopt(cuda, oracle_mod, layout):
    """Store mode on the var tile loop: a load that starts in the header window and ends past
    byte 64 reads its low bytes from the window in LDS (stored ones included) and its high bytes
    from the overflow image (lanes that stored there) or the packet (zeros at or past LEN) --
    jit.cpp ldx_fixed -- instead of deoptimizing: the deopt pass re-runs no packet, and every
    output == the general interpreter's == the oracle's. Packets of 0..100 bytes, so LEN falls
    inside, before and after the straddled bytes."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu.asm import assemble
    from test_stack_tier import VAR_LAYOUTS, _fixed_frames, _images_of

    img = assemble(STRADDLE_PROG)
    rng = random.Random(99 + len(layout))
    pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 15, 16, 40, 60, 64, 65, 66, 68,
                                                                  70, 71, 72, 80, 100])))
            for _ in range(3000)]
    prog = Program(img)
    assert prog.store_mode
    if layout.startswith("fixed"):
        stride = int(layout[5:])
        pk = [p[:stride].ljust(stride, b"\0") for p in pkts]
        frames = _fixed_frames(pk, stride, cuda)
        kw = dict(n=len(pk), stride=stride)
        xdp = False
    else:
        from test_gpu_parity import _stage

        spec = dict(VAR_LAYOUTS[layout])
        xdp = spec.pop("xdp", False)
        pk = pkts
        frames, kw = _stage(pkts, cuda, **spec)
    b = prog.make_batch(frames, xdp_md=xdp, **kw)
    ws = torch.zeros(prog.workspace_bytes(b, 0), dtype=torch.uint8, device=cuda)
    b = prog.make_batch(frames, xdp_md=xdp, workspace=ws, **kw)
    assert prog.batch_kernel(b) in (_lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK)
    out = _lib.BatchOut()
    r0 = torch.empty(len(pk), dtype=torch.int64, device=cuda)
    st = torch.empty(len(pk), dtype=torch.uint8, device=cuda)
    ws[8:12] = 0xFF
    out.r0, out.status = r0.data_ptr(), st.data_ptr()
    prog.launch(b, out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    _assert_no_deopt(ws, prog)
    gen = prog.run(frames, r0=True, status=True, generic=True, xdp_md=xdp, **kw)
    torch.cuda.synchronize()
    assert torch.equal(st, gen.status)
    ok = st == 0
    assert torch.equal(r0[ok], gen.r0[ok])
    op = oracle_mod.Program(img)
    stn, r0n = st.cpu().numpy(), r0.cpu().numpy().view(np.uint64)
    for i, im in enumerate(_images_of(pk, xdp)):
        s, o0, _ = op.run_packet(im, 1024, 512, 1 << 22)
        assert stn[i] == s, (layout, i)
        if s == 0:
            assert int(r0n[i]) == o0, (layout, i)
    prog.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed128", "offsets_mis3"])
def test_no_deopt_proof_fuzz(cuda, oracle_mod, layout):
    """Store-mode programs that jit.cpp store_mode_no_deopt proves deopt-free (every
    register-address store ends at or below byte 128, and -- when one may pass byte 64 -- every
    register-address load too, no constant-address load past 64) run on the var tile loop without
    the deopt pass. A wrong proof would leave listed lanes without outputs, so: the list stays
    empty, the pass is not launched, and every output == the general interpreter's == the
    oracle's. Also: the same program with r10 below 128 + the stack window keeps its pass."""
    import torch

    from ebpf_emu import Program, _lib
    from test_stack_tier import VAR_LAYOUTS, _fixed_frames, _images_of, _var_packets

    rng = random.Random(zlib.crc32(b"proof" + layout.encode()))
    done = nopass = 0
    for it in range(160):
        img = gen_store_program(rng)
        try:
            oracle_mod.Program(img)
            prog = Program(img)
        except Exception:
            continue
        if not (prog.store_mode and prog.store_mode_no_deopt):
            prog.close()
            continue
        pkts = _var_packets(rng, rng.choice([64, 100, 130]))
        if layout.startswith("fixed"):
            pk = [p[:128].ljust(128, b"\0") for p in pkts]
            frames = _fixed_frames(pk, 128, cuda)
            kw = dict(n=len(pk), stride=128)
        else:
            from test_gpu_parity import _stage

            pk = pkts
            frames, kw = _stage(pkts, cuda, **VAR_LAYOUTS[layout])
        for r10 in (512, 100):
            b = prog.make_batch(frames, r10=r10, **kw)
            if prog.batch_kernel(b) not in (_lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK):
                break
            ws = torch.zeros(prog.workspace_bytes(b, 0), dtype=torch.uint8, device=cuda)
            b = prog.make_batch(frames, r10=r10, workspace=ws, **kw)
            out = _lib.BatchOut()
            r0 = torch.empty(len(pk), dtype=torch.int64, device=cuda)
            st = torch.empty(len(pk), dtype=torch.uint8, device=cuda)
            ws[8:12] = 0xFF
            out.r0, out.status = r0.data_ptr(), st.data_ptr()
            prog.launch(b, out, torch.cuda.current_stream())
            torch.cuda.synchronize()
            w = ws[:12].cpu().numpy().view(np.uint32)
            if r10 == 512:  # (the stack window at 512 - k: no lane deoptimizes; no pass when the
                            # stores' bound -- or mem_size -- ends before it)
                assert w[0] == 0 and w[2] in (0, 0xFFFFFFFF), (it, w, img.hex())
                nopass += w[2] == 0xFFFFFFFF
            else:  # (r10 - k below 128: the pass runs)
                assert w[0] == 0 and w[2] != 0xFFFFFFFF, (it, w, img.hex())
            gen = prog.run(frames, r0=True, status=True, generic=True, r10=r10, **kw)
            torch.cuda.synchronize()
            assert torch.equal(st, gen.status), (it, r10, img.hex())
            ok = st == 0
            assert torch.equal(r0[ok], gen.r0[ok]), (it, r10, img.hex())
            if r10 == 512:
                op = oracle_mod.Program(img)
                stn, r0n = st.cpu().numpy(), r0.cpu().numpy().view(np.uint64)
                for i, im in enumerate(_images_of(pk, False)):
                    s, o0, _ = op.run_packet(im, 1024, 512, 1 << 22)
                    assert stn[i] == s, (it, i)
                    if s == 0:
                        assert int(r0n[i]) == o0, (it, i)
        else:
            done += 1
        prog.close()
    assert done >= 8 and nopass >= 4, (done, nopass)
