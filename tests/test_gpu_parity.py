"""HIP-kernel parity on an MI355X, through the C ABI (libebpfemu.so), against the C oracle and
the committed golden fixtures. Bit-exact: status for every packet; r0, all registers and the
whole memory image for every packet that completes."""
import json
import os
import random
import zlib

import numpy as np
import pytest

from cases import CASES
from fuzzgen import gen_packet, gen_program

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STEPS = 20000  # step budget used on both sides


def _torch():
    import torch

    return torch


def _stage(pkts, dev, stride=None, offsets_layout=False, misalign=0, align=1):
    """Pack packets into one device buffer. Returns (frames, kwargs for Program.run)."""
    torch = _torch()
    lens = np.array([len(p) for p in pkts], dtype=np.uint16)
    if offsets_layout:
        offs, pos, chunks = [], 0, []
        for p in pkts:
            pad = misalign + (-(pos + misalign)) % align
            pos += pad
            chunks.append(bytes(pad))
            offs.append(pos)
            chunks.append(p)
            pos += len(p)
        buf = b"".join(chunks) + bytes(16)
        frames = torch.tensor(np.frombuffer(buf, dtype=np.uint8).copy(), device=dev)
        o = torch.tensor(np.array(offs, dtype=np.uint32).view(np.int32), device=dev)
        ln = torch.tensor(lens.view(np.int16), device=dev)
        return frames, dict(n=len(pkts), offsets=o, lens=ln)
    stride = stride or max(64, max((len(p) for p in pkts), default=0) + 15) // 16 * 16
    buf = np.zeros(len(pkts) * stride, dtype=np.uint8)
    for i, p in enumerate(pkts):
        buf[i * stride:i * stride + len(p)] = np.frombuffer(p, dtype=np.uint8)
    frames = torch.tensor(buf, device=dev)
    ln = torch.tensor(lens.view(np.int16), device=dev)
    return frames, dict(n=len(pkts), stride=stride, lens=ln)


_PROG = {}  # the last image's loaded program, shared by its full, generic and production runs


def _shared(img):
    from ebpf_emu import Program

    if img not in _PROG:
        for q in _PROG.values():
            q.close()
        _PROG.clear()
        _PROG[img] = Program(img)
    return _PROG[img]


def _run_full(prog_img, pkts, dev, mem_size=1024, r10=512, max_steps=STEPS, generic=False,
              **layout):
    torch = _torch()
    prog = _shared(prog_img)
    frames, kw = _stage(pkts, dev, **layout)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    res = prog.run(frames, mem_size=mem_size, r10=r10, max_steps=max_steps, verdict=True, r0=True,
                   status=True, mem=True, regs=True, counters=cnt, generic=generic, **kw)
    torch.cuda.synchronize()
    out = dict(status=res.status.cpu().numpy(), r0=res.r0.cpu().numpy().view(np.uint64),
               verdict=res.verdict.cpu().numpy(), regs=res.regs.cpu().numpy().view(np.uint64),
               mem=res.mem.cpu().numpy(), counters=cnt.cpu().numpy().view(np.uint64),
               tier=prog.tier, fast=prog.forward_only and not generic and max_steps >= len(prog))
    return out


def _run_prod(prog_img, pkts, dev, mem_size=1024, r10=512, max_steps=STEPS, **layout):
    """The outputs a production caller asks for (bench.py, pcap.py): no registers, no image, so
    the kernels take their production paths -- the compiled programs' liveness-pruned register
    init (jit.cpp live_in, ;@@JITINIT@@) and, for a verdict-only launch, the k_flags = 0 epilogue.
    Two launches: verdict + counters only, then r0 + status (still without registers)."""
    torch = _torch()
    prog = _shared(prog_img)
    frames, kw = _stage(pkts, dev, **layout)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    v = prog.run(frames, mem_size=mem_size, r10=r10, max_steps=max_steps, verdict=True,
                 counters=cnt, **kw)
    rs = prog.run(frames, mem_size=mem_size, r10=r10, max_steps=max_steps, verdict=False,
                  r0=True, status=True, **kw)
    torch.cuda.synchronize()
    out = dict(verdict=v.verdict.cpu().numpy(), counters=cnt.cpu().numpy().view(np.uint64),
               r0=rs.r0.cpu().numpy().view(np.uint64), status=rs.status.cpu().numpy())
    return out


def _check_prod_against_oracle(oracle_mod, img, pkts, got, mem_size=1024, r10=512, tag="",
                               max_steps=STEPS):
    op = oracle_mod.Program(img)
    cnt = np.zeros(8, dtype=np.uint64)
    for i, p in enumerate(pkts):
        st, r0, steps = op.run_packet(p, mem_size, r10, max_steps)
        ctx = f"{tag} pkt {i} prog {img.hex()} pkt {p.hex()}"
        assert got["status"][i] == st, ctx
        if st == 0:
            assert int(got["r0"][i]) == r0, ctx
            v = r0 if r0 < 5 else 0xFE
            cnt[r0 if r0 < 5 else 5] += 1
        else:
            v = 0xFF
            cnt[6] += 1
        assert got["verdict"][i] == v, ctx
        cnt[7] += steps
    assert list(got["counters"]) == list(cnt), tag


def _check_against_oracle(oracle_mod, img, pkts, got, mem_size=1024, r10=512, tag=""):
    op = oracle_mod.Program(img)
    cnt = np.zeros(8, dtype=np.uint64)
    for i, p in enumerate(pkts):
        st, regs, mem, steps = op.run_full(p, mem_size, r10, STEPS)
        ctx = f"{tag} pkt {i} prog {img.hex()} pkt {p.hex()}"
        assert got["status"][i] == st, ctx
        if st == 0:
            assert int(got["r0"][i]) == regs[0], ctx
            assert [int(v) for v in got["regs"][i]] == regs, ctx
            assert bytes(got["mem"][i]) == mem, ctx
            v = regs[0] if regs[0] < 5 else 0xFE
            cnt[regs[0] if regs[0] < 5 else 5] += 1
        else:
            v = 0xFF
            cnt[6] += 1
        assert got["verdict"][i] == v, ctx
        cnt[7] += steps
    assert list(got["counters"]) == list(cnt), tag


def test_directed_cases(cuda, oracle_mod):
    for c in CASES:
        got = _run_full(c.prog, [c.pkt], cuda, c.mem_size, c.r10, max_steps=c.max_steps or STEPS)
        assert got["status"][0] == c.status, c.name
        if c.status == 0:
            assert int(got["r0"][0]) == c.r0, c.name
        # the oracle with the same budget agrees on everything observable
        op = oracle_mod.Program(c.prog)
        st, regs, mem, steps = op.run_full(c.pkt, c.mem_size, c.r10, c.max_steps or STEPS)
        assert st == got["status"][0], c.name
        if st == 0:
            assert [int(v) for v in got["regs"][0]] == regs, c.name
            assert bytes(got["mem"][0]) == mem, c.name


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_wave_divergence(cuda, oracle_mod, seed):
    """Random programs, each over 64..130 random packets in one batch: lanes diverge on packet
    contents, fault at different steps, loop into the budget, mix both memory tiers."""
    rng = random.Random(4242 + seed)
    tiers = set()
    for it in range(60):
        img = gen_program(rng)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        pkts = [gen_packet(rng) for _ in range(rng.choice([64, 65, 100, 130]))]
        got = _run_full(img, pkts, cuda)
        tiers.add(got["tier"])
        _check_against_oracle(oracle_mod, img, pkts, got, tag=f"seed {seed} it {it}")
        # the production outputs (no registers / image): the same program and packets
        prod = _run_prod(img, pkts, cuda)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, tag=f"prod seed {seed} it {it}")
    assert tiers == {0, 1}


_OUT_KEYS = ("status", "r0", "verdict", "regs", "mem", "counters")


def _same_outputs(a, b, ctx):
    for key in _OUT_KEYS:
        assert np.array_equal(a[key], b[key]), f"{ctx}: {key} differs"


@pytest.mark.parametrize("seed", range(4))
def test_forward_only_fast_path_fuzz(cuda, oracle_mod, seed):
    """Forward-only tier-0 programs (the dag_kernel fast path) over diverging packets: every
    output bit-identical to the general interpreter on the same batch (EBPF_BATCH_GENERIC) and
    to the oracle."""
    rng = random.Random(9000 + seed)
    n_fast = 0
    for it in range(50):
        img = gen_program(rng, allow_loops=False, tier0=True)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        pkts = [gen_packet(rng) for _ in range(rng.choice([64, 65, 100, 130]))]
        got = _run_full(img, pkts, cuda)
        assert got["fast"], img.hex()
        n_fast += 1
        ref = _run_full(img, pkts, cuda, generic=True)
        _same_outputs(got, ref, f"seed {seed} it {it} prog {img.hex()}")
        _check_against_oracle(oracle_mod, img, pkts, got, tag=f"seed {seed} it {it}")
        prod = _run_prod(img, pkts, cuda)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, tag=f"prod seed {seed} it {it}")
    assert n_fast >= 35


@pytest.mark.parametrize("pad", [40, 120, 230])
def test_forward_only_wide_pc_set(cuda, oracle_mod, pad):
    """Fast-path programs past 64 micro-ops (four-word pc set): forward jumps over `pad` filler
    instructions, some of which are executed by the lanes that take the other branch."""
    from ebpf_emu.asm import assemble

    rng = random.Random(77 + pad)
    for it in range(6):
        body = gen_program(rng, n=20, allow_loops=False, tier0=True)
        head = assemble(f"ldxb r3, [r1+0]\njgt r3, 127, +{pad}\n" + "add r0, 3\n" * pad)
        img = head + body
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        pkts = [gen_packet(rng) for _ in range(97)]
        got = _run_full(img, pkts, cuda)
        assert got["fast"]
        _same_outputs(got, _run_full(img, pkts, cuda, generic=True), f"pad {pad} it {it}")
        _check_against_oracle(oracle_mod, img, pkts, got, tag=f"pad {pad} it {it}")


CONST_LOAD_PROGRAMS = [
    "mov r1, 8\nldxb r0, [r1+2]\nexit",                                   # rebased constant
    "jeq r2, 60, +2\nmov r1, 4\nja +1\nmov r1, 6\nldxb r0, [r1+0]\nexit",  # join, differs
    "jeq r2, 60, +2\nmov r1, 4\nja +1\nmov r1, 4\nldxh r0, [r1+1]\nexit",  # join, agrees
    "lddw r1, 0x7fffffffffffffff\nldxb r0, [r1+1]\nexit",                # static overflow
    "add r1, 20\nldxw r0, [r1+3]\nexit",                                  # add on a constant
    "mov r1, r2\nldxb r0, [r1-1]\nexit",                                  # per-lane: not folded
    "ldxdw r0, [r1+60]\nldxb r3, [r1+70]\nadd r0, r3\nexit",               # past the window
    "ldxb r0, [r1+1023]\nldxh r3, [r1+1023]\nexit",                         # image end, tail UB
    "ldxb r0, [r1-1]\nexit",                                               # negative address
    "mov32 r1, -1\nldxb r0, [r1+0]\nexit",                                # zero-extended mov32
    "ldxw r1, [r1+0]\nldxb r0, [r1+0]\nexit",                             # base from a load
]


def test_forward_only_constant_address_loads(cuda, oracle_mod):
    """Loads whose base register is a load-time constant (resolved addresses on the fast path)
    at the edges of the dataflow: joins, overflow, window/image ends, non-constant bases."""
    from ebpf_emu.asm import assemble

    rng = random.Random(5)
    pkts = [bytes(rng.getrandbits(8) for _ in range(n))
            for n in (0, 1, 3, 14, 60, 63, 64, 65, 70, 71, 200, 1024)]
    pkts += [gen_packet(rng) for _ in range(60)]
    for src in CONST_LOAD_PROGRAMS:
        img = assemble(src)
        got = _run_full(img, pkts, cuda)
        assert got["fast"], src
        _same_outputs(got, _run_full(img, pkts, cuda, generic=True), src)
        _check_against_oracle(oracle_mod, img, pkts, got, tag=src)


def test_forward_only_step_budget_falls_back(cuda, oracle_mod):
    """max_steps below the program length can bind, so the batch runs on the general
    interpreter: same statuses as the oracle with that budget."""
    from ebpf_emu.asm import assemble

    img = assemble("mov r0, 1\n" * 10 + "exit")
    pkts = [bytes(range(n)) for n in (0, 5, 64, 70)]
    for budget in (1, 5, 10, 11, 12):
        got = _run_full(img, pkts, cuda, max_steps=budget)
        assert got["fast"] == (budget >= 11)
        op = oracle_mod.Program(img)
        for i, p in enumerate(pkts):
            st, regs, mem, steps = op.run_full(p, 1024, 512, budget)
            assert got["status"][i] == st, (budget, i)
            if st == 0:
                assert [int(v) for v in got["regs"][i]] == regs


@pytest.mark.parametrize("pad", [70, 300, 5000])
def test_program_size_variants(cuda, oracle_mod, pad):
    """Programs past 64 / 256 micro-ops (wider pc-set scheduler, DPP wave-min scheduler) and past
    4096 (micro-ops fetched from global memory instead of LDS): a `ja` over `pad` never-executed
    instructions, then a fuzzed program; some programs also jump back into the padding."""
    from ebpf_emu.asm import encode

    rng = random.Random(77 + pad)
    filler = b"".join(encode(0xB7, rng.randrange(10), 0, 0, rng.randrange(100)) for _ in range(pad))
    n_ok = 0
    for it in range(25):
        body = gen_program(rng)
        try:
            oracle_mod.Program(body)
        except oracle_mod.OracleDecodeError:
            continue
        img = encode(0x05, 0, 0, pad) + filler + body
        if it % 5 == 0:  # re-enter the padding from the end of the program
            img += encode(0x05, 0, 0, -(len(img) // 8) + 1 + rng.randrange(pad))
        pkts = [gen_packet(rng) for _ in range(70)]
        got = _run_full(img, pkts, cuda)
        _check_against_oracle(oracle_mod, img, pkts, got, tag=f"pad {pad} it {it}")
        n_ok += 1
    assert n_ok >= 15


def test_layouts_and_alignment(cuda, oracle_mod):
    """Stride and offsets layouts, 16-byte-aligned (coalesced staging) and misaligned (per-lane
    staging) packet bases, packets shorter/longer than the 64-byte LDS window."""
    from ebpf_emu import workloads as W

    rng = random.Random(99)
    pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 13, 34, 63, 64, 65, 100, 200])))
            for _ in range(300)]
    for name in ("5tuple", "checksum", "drop"):
        img = W.program(name)
        for layout in (dict(), dict(stride=208), dict(offsets_layout=True, align=16),
                       dict(offsets_layout=True), dict(offsets_layout=True, misalign=3),
                       dict(offsets_layout=True, misalign=1, align=16)):
            got = _run_full(img, pkts, cuda, **layout)
            _check_against_oracle(oracle_mod, img, pkts, got, tag=f"{name} {layout}")


def test_large_image_and_stack(cuda, oracle_mod):
    """mem_size 2048 / r10 2048 (the mixed-frame layout) and a small 64-byte image."""
    rng = random.Random(5)
    for mem_size, r10 in ((2048, 2048), (64, 64), (1024, 512)):
        for it in range(15):
            img = gen_program(rng)
            try:
                oracle_mod.Program(img)
            except oracle_mod.OracleDecodeError:
                continue
            pkts = [gen_packet(rng, max_len=min(80, mem_size + 8)) for _ in range(70)]
            got = _run_full(img, pkts, cuda, mem_size=mem_size, r10=r10)
            _check_against_oracle(oracle_mod, img, pkts, got, mem_size=mem_size, r10=r10,
                                  tag=f"mem {mem_size} it {it}")


def test_golden_fuzz_vectors(cuda):
    """Committed fixtures (tests/golden/fuzz_vectors.json): no oracle at run time."""
    with open(os.path.join(GOLDEN, "fuzz_vectors.json")) as f:
        g = json.load(f)
    for v in g["vectors"]:
        img = bytes.fromhex(v["prog"])
        pkts = [bytes.fromhex(p) for p in v["pkts"]]
        got = _run_full(img, pkts, cuda, max_steps=g["max_steps"])
        for i, e in enumerate(v["expect"]):
            assert got["status"][i] == e["status"], (v["prog"], i)
            if e["status"] == 0:
                assert int(got["r0"][i]) == int(e["r0"], 16)
                assert zlib.crc32(bytes(got["mem"][i])) == e["mem_crc32"]
                assert [int(x) for x in got["regs"][i]] == [int(r, 16) for r in e["regs"]]


@pytest.mark.parametrize("config", ["drop", "5tuple", "checksum"])
def test_workload_golden_full_size(cuda, config):
    """BASELINE configs 2/3/5 at full size (1M packets): counters and the CRC of the verdict
    array equal the committed fixture (generated by the oracle, tests/golden/make_golden.py)."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    with open(os.path.join(GOLDEN, "workloads.json")) as f:
        g = json.load(f)[config]
    prog = Program(W.program(config))
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    if g["layout"] == "fixed":
        buf = W.frames_fixed(g["n"], 64, g["config_id"])
        frames = torch.from_numpy(buf).to(cuda)
        res = prog.run(frames, n=g["n"], stride=64, counters=cnt)
    else:
        buf, offs, lens = W.frames_mixed(g["n"], config_id=g["config_id"])
        frames = torch.from_numpy(buf).to(cuda)
        res = prog.run(frames, n=g["n"], offsets=torch.from_numpy(offs.view(np.int32)).to(cuda),
                       lens=torch.from_numpy(lens.view(np.int16)).to(cuda), mem_size=g["mem_size"],
                       r10=g["r10"], counters=cnt)
    torch.cuda.synchronize()
    verdict = res.verdict.cpu().numpy()
    assert [int(x) for x in cnt.cpu().numpy().view(np.uint64)] == g["counters"]
    assert zlib.crc32(verdict.tobytes()) == g["verdict_crc32"]
    assert verdict[:256].tolist() == g["verdict_head"]
    # size-independent property: every packet lands in exactly one bucket
    assert int(cnt[:7].sum()) == g["n"]


def test_workload_sample_vs_oracle(cuda, oracle_mod):
    """64Ki-packet samples of each workload, per packet vs the oracle batch."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    n = 65536 + 37  # ragged tail
    buf = W.frames_fixed(n, 64, 3)
    frames = torch.from_numpy(buf).to(cuda)
    for name in ("drop", "5tuple", "acl"):
        prog = Program(W.program(name))
        res = prog.run(frames, n=n, stride=64, r0=True, status=True)
        torch.cuda.synchronize()
        r0, st, _ = oracle_mod.Program(W.program(name)).run_batch(buf, n, stride=64, threads=8)
        assert np.array_equal(res.status.cpu().numpy(), st)
        assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), r0)
    buf, offs, lens = W.frames_mixed(4096 + 5, config_id=5)
    prog = Program(W.program("checksum"))
    res = prog.run(torch.from_numpy(buf).to(cuda), n=len(offs),
                   offsets=torch.from_numpy(offs.view(np.int32)).to(cuda),
                   lens=torch.from_numpy(lens.view(np.int16)).to(cuda), mem_size=2048, r10=2048,
                   r0=True, status=True)
    torch.cuda.synchronize()
    r0, st, _ = oracle_mod.Program(W.program("checksum")).run_batch(
        buf, len(offs), offsets=offs, lens=lens, mem_size=2048, r10=2048, threads=8)
    assert np.array_equal(res.status.cpu().numpy(), st)
    assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), r0)


def test_tier1_workload_vs_oracle(cuda, oracle_mod):
    """The tier-1 bench workload (workloads.MAC_SWAP_TX: packet stores, a stack atomic) on 64 Ki
    + 5 fixed-slot frames -- on the compiled kernel (memory tier 0.5 with packet-window stores)
    and on the general interpreter (tier 1): status, r0 and counters equal the oracle's, and the
    final images of a sample (an image output: the general interpreter) show the swapped MACs."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    n = 65536 + 5
    buf = W.frames_fixed(n, 64, 3)
    frames = torch.from_numpy(buf).to(cuda)
    img = W.program("mac_swap_tx")
    prog = Program(img)
    r0, st, ocnt = oracle_mod.Program(img).run_batch(buf, n, stride=64, threads=8)
    assert int(ocnt[3]) == n  # every 64-byte frame reflected
    for generic, kernel in ((False, _lib.EBPF_KERNEL_JIT_STACK), (True, _lib.EBPF_KERNEL_GENERAL_T1)):
        assert prog.batch_kernel(prog.make_batch(frames, n=n, stride=64, generic=generic)) == kernel
        cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
        res = prog.run(frames, n=n, stride=64, r0=True, status=True, counters=cnt, generic=generic)
        torch.cuda.synchronize()
        assert np.array_equal(res.status.cpu().numpy(), st), generic
        assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), r0), generic
        assert np.array_equal(cnt.cpu().numpy().view(np.uint64), ocnt), generic
    pk = [bytes(buf[i * 64:(i + 1) * 64]) for i in range(64)]
    got = _run_full(img, pk, cuda, stride=64)
    _check_against_oracle(oracle_mod, img, pk, got, tag="mac swap")
    assert bytes(got["mem"][0][:12]) == pk[0][6:12] + pk[0][0:6]


def test_counters_accumulate_and_caller_workspace(cuda):
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    n = 10000
    frames = torch.from_numpy(W.frames_fixed(n, 64, 3)).to(cuda)
    prog = Program(W.program("5tuple"))
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    prog.run(frames, n=n, stride=64, counters=cnt)
    once = cnt.clone()
    b = prog.make_batch(frames, n=n, stride=64)
    ws = torch.zeros(prog.workspace_bytes(b, 0), dtype=torch.uint8, device=cuda)
    prog.run(frames, n=n, stride=64, counters=cnt)
    torch.cuda.synchronize()
    assert torch.equal(cnt, 2 * once)
    b = prog.make_batch(frames, n=n, stride=64, workspace=ws)
    from ebpf_emu import _lib

    out = _lib.BatchOut()
    out.counters = cnt.data_ptr()
    prog.launch(b, out)
    torch.cuda.synchronize()
    assert torch.equal(cnt, 3 * once)


def test_emu_api_init_regs(cuda):
    """The reference's Emu surface (emu.rs:19-45,452): caller-set registers and memory."""
    from ebpf_emu import Emu, EmuPanic
    from ebpf_emu.asm import assemble
    from ebpf_emu.ins import hexs_to_instructions
    from ebpf_emu.mmu import Mmu

    emu = Emu()
    emu.state.mmu = Mmu(bytearray(1024))
    emu.state.mmu.memory[:5] = bytes.fromhex("aabbffccdd")
    emu.state.regs[2] = 5
    emu.state.regs[10] = 512
    emu.instructions = hexs_to_instructions(
        "b4 02 00 00 11 00 00 00 73 21 02 00 00 00 00 00 71 10 02 00 00 00 00 00 95 00 00 00 00 00 00 00")
    emu.run()
    assert emu.state.regs[0] == 0x11
    assert emu.state.mmu.memory[2] == 0x11
    emu = Emu()
    emu.state.mmu = Mmu(bytearray(64))
    emu.state.regs[3] = 7
    emu.state.regs[4] = -3
    from ebpf_emu.ins import decode_image

    emu.instructions = decode_image(assemble("mov r0, r3\nadd r0, r4\nexit"))
    emu.run()
    assert emu.state.regs[0] == 4
    emu.instructions = decode_image(assemble("ldxb r0, [r1+64]\nexit"))
    with pytest.raises(EmuPanic):
        emu.run()


def test_emem_cli_kats(cuda):
    """The emem plugin protocol (main.rs:5-44) end to end on the GPU."""
    import subprocess

    emem = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ebpf-emu_amd", "bin", "emem")
    kat1 = "b7 00 00 00 00 00 00 00 17 00 00 00 01 00 00 00 74 00 00 00 08 00 00 00 95 00 00 00 00 00 00 00"
    r = subprocess.run([emem, ""], input=kat1 + "\n", capture_output=True, text=True, timeout=120)
    assert (r.returncode, r.stdout) == (0, "ffffff\n"), r.stderr
    r = subprocess.run([emem, "", kat1], input="", capture_output=True, text=True, timeout=120)
    assert (r.returncode, r.stdout) == (0, "ffffff\n"), r.stderr
    prog = "b7 00 00 00 ff ff ff ff 95 00 00 00 00 00 00 00"  # mov r0, -1 -> two's complement hex
    r = subprocess.run([emem, ""], input=prog + "\n", capture_output=True, text=True, timeout=120)
    assert r.stdout == "ffffffffffffffff\n"
    memlen = "bf 20 00 00 00 00 00 00 95 00 00 00 00 00 00 00"  # mov r0, r2 (mem-len)
    r = subprocess.run([emem, "aa bb cc"], input=memlen + "\n", capture_output=True, text=True, timeout=120)
    assert r.stdout == "3\n"
    r = subprocess.run([emem, ""], input="71 10 00 04 00 00 00 00 95 00 00 00 00 00 00 00\n",
                       capture_output=True, text=True, timeout=120)  # ldxb r0, [r1+1024] -> panic
    assert r.returncode == 101


def test_conformance_runner(cuda):
    """The `.data` runner over the reference-derived vectors, through the GPU path."""
    import os

    from ebpf_emu.conformance import main

    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "conformance")
    assert main([d]) == 0


@pytest.mark.timeout(600)
def test_config4_global_batch_golden(cuda):
    """BASELINE config 4: the 5-tuple over the 100,000,000-packet global batch (seeded 1 Mi-packet
    chunks, bench.py --total-packets) as ONE batch on one GPU -- the strong-scaling workload every
    rank count must reproduce. Counters and every chunk's verdict CRC32 equal the committed
    fixture (tests/golden/make_golden.py config4, from the oracle)."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    from ebpf_emu import Program
    from ebpf_emu import dist as D

    with open(os.path.join(GOLDEN, "config4.json")) as f:
        g = json.load(f)
    sizes = g["chunk_sizes"]
    n = g["total_packets"]
    assert sum(sizes) == n
    frames = torch.empty(n * 64, dtype=torch.uint8, device=cuda)
    starts = np.concatenate([[0], np.cumsum(sizes)])

    def put(k):
        return k, D.chunk_frames(k, sizes[k])

    with ThreadPoolExecutor(8) as ex:  # host generation in threads, copies in order
        for k, buf in ex.map(put, range(len(sizes))):
            frames[int(starts[k]) * 64:int(starts[k + 1]) * 64].copy_(torch.from_numpy(buf))
    prog = Program(bytes.fromhex(g["program"]))
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    res = prog.run(frames, n=n, stride=64, counters=cnt)
    torch.cuda.synchronize()
    verdict = res.verdict.cpu().numpy()
    assert [int(x) for x in cnt.cpu().numpy().view(np.uint64)] == g["counters"]
    for k in range(len(sizes)):
        v = verdict[int(starts[k]):int(starts[k + 1])]
        assert zlib.crc32(v.tobytes()) == g["chunk_verdict_crc32"][k], k
        assert np.bincount(v, minlength=256)[1] == g["chunk_counters"][k][1], k
    del frames, res
    prog.close()


def test_run_batch_multi_single_shard(cuda):
    """ebpf_run_batch_multi with one shard on device 0 (the RCCL counter all-reduce over a
    one-rank communicator) equals ebpf_run_batch: the same verdicts, and the counters ADDED to
    the caller's (accumulated, as the header promises), twice in a row."""
    import ctypes

    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    n = 300_001
    frames = torch.from_numpy(W.frames_fixed(n, 64, 3)).to(cuda)
    prog = Program(W.program("5tuple"))
    ref_cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    ref = prog.run(frames, n=n, stride=64, counters=ref_cnt)
    torch.cuda.synchronize()
    b = prog.make_batch(frames, n=n, stride=64)
    verdict = torch.empty(n, dtype=torch.uint8, device=cuda)
    cnt = torch.full((8,), 7, dtype=torch.int64, device=cuda)  # caller's running totals
    out = _lib.BatchOut()
    out.verdict = verdict.data_ptr()
    out.counters = cnt.data_ptr()
    stream = torch.cuda.current_stream(cuda)
    devs = (ctypes.c_int * 1)(0)
    batches = (_lib.Batch * 1)(b)
    outs = (_lib.BatchOut * 1)(out)
    streams = (ctypes.c_void_p * 1)(stream.cuda_stream)
    L = _lib.lib()
    for rep in (1, 2):
        rc = L.ebpf_run_batch_multi(prog._h, 1, devs, batches, outs, streams)
        assert rc == 0, _lib.strerror(rc)
        torch.cuda.synchronize()
        assert torch.equal(verdict, ref.verdict)
        assert cnt.cpu().tolist() == [7 + rep * int(c) for c in ref_cnt.cpu().tolist()]
    # a repeated device is rejected before anything runs
    devs2 = (ctypes.c_int * 2)(0, 0)
    assert L.ebpf_run_batch_multi(prog._h, 2, devs2, (_lib.Batch * 2)(b, b),
                                  (_lib.BatchOut * 2)(out, out),
                                  (ctypes.c_void_p * 2)(stream.cuda_stream, stream.cuda_stream)) \
        == _lib.EBPF_EINVAL
    prog.close()


def test_emu_any_image_length_and_frame_stack(cuda, oracle_mod):
    """The Emu surface beyond the main.rs layout: an image of any length (Mmu.memory: Vec<u8>,
    mmu.rs:2-4) with loads at its last bytes, and the pub frame stack Emu.fp (emu.rs:26) -- an
    initial stack popped by EXIT (emu.rs:273-279), and a program that falls off its end inside a
    call leaving a non-empty stack. Every case against the oracle's run_image."""
    from ebpf_emu import Emu, EmuPanic
    from ebpf_emu.asm import assemble
    from ebpf_emu.ins import decode_image
    from ebpf_emu.mmu import Mmu

    cases = [
        ("ldxb r0, [r1+12]\nexit", bytes(range(1, 14)), (), [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0]),
        ("ldxh r0, [r1+12]\nexit", bytes(range(1, 14)), (), [0] * 11),       # tail past the end
        ("ldxw r0, [r1+9]\nexit", bytes(range(1, 14)), (), [0] * 11),
        ("stb [r1+4], 0x77\nldxdw r0, [r1+0]\nexit", bytes(range(1, 10)), (), [0] * 11),
        ("mov r0, 5\nexit", b"", (), [0] * 11),                              # empty image
        ("ldxb r0, [r1+0]\nexit", b"", (), [0] * 11),                        # ... faults
        ("mov r0, 1\nexit\nmov r0, 2\nexit", bytes(3), (2,), [0] * 11),      # EXIT pops fp
        ("mov r0, 1\nexit\nmov r0, 2\nexit", bytes(3), (2, 3), [0] * 11),    # pops to pc 3
        ("mov r0, 1\nexit", bytes(5), (1000,), [0] * 11),                    # pops past the end
        ("call 1\nexit\nmov r0, 9", bytes(7), (), [0] * 11),                 # falls off in a call
        ("call 1\nexit\nmov r0, 9", bytes(7), (5, 6), [0] * 11),
        ("add r0, r3\nexit", bytes(11), (), [1, 0, 0, 41, 0, 0, 0, 0, 0, 0, 0]),
    ]
    for src, image, fp, regs in cases:
        img = assemble(src)
        st, oregs, omem, ofp, _ = oracle_mod.Program(img).run_image(image, regs, fp, 20000)
        emu = Emu()
        emu.state.mmu = Mmu(bytearray(image))
        emu.state.regs = list(regs)
        emu.fp = list(fp)
        emu.instructions = decode_image(img)
        if st == 0:
            emu.run()
            assert [r & ((1 << 64) - 1) for r in emu.state.regs] == oregs, src
            assert bytes(emu.state.mmu.memory) == omem, src
            assert emu.fp == ofp, (src, fp)
        else:
            with pytest.raises(EmuPanic) as e:
                emu.run()
            assert e.value.status == st, src


@pytest.mark.parametrize("config", ["5tuple", "checksum"])
@pytest.mark.parametrize("own_ws", [True, False])
def test_concurrent_streams(cuda, config, own_ws):
    """Consecutive batches on two streams (bench.py --streams 2): launches alternate over two
    streams that run at once, each with its own workspace (explicit, or the library's per-stream
    one) and verdict buffer, all folding into ONE counters array. Every stream's verdicts equal a
    one-stream run's, and the shared counters equal the sum of the one-stream runs."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    n = 1 << 16
    prog = Program(W.program(config))
    prog.upload(0)
    keep = []  # (the device buffers the batch descriptors point into)
    descs = []
    for k in range(3):
        if config == "checksum":
            b, o, ln = W.frames_mixed(n, config_id=5 + 100 * k)
            t = [torch.from_numpy(b).to(cuda), torch.from_numpy(o.view(np.int32)).to(cuda),
                 torch.from_numpy(ln.view(np.int16)).to(cuda)]
            descs.append(prog.make_batch(t[0], n=n, offsets=t[1], lens=t[2], mem_size=2048,
                                         r10=2048))
        else:
            t = [torch.from_numpy(W.frames_fixed(n, 64, 3 + 100 * k)).to(cuda)]
            descs.append(prog.make_batch(t[0], n=n, stride=64, mem_size=1024, r10=512))
        keep += t
    # one stream, one batch at a time: the reference verdicts and counters
    ref_v, ref_c = [], []
    for d in descs:
        v = torch.empty(n, dtype=torch.uint8, device=cuda)
        c = torch.zeros(8, dtype=torch.int64, device=cuda)
        o = _lib.BatchOut()
        o.verdict, o.counters = v.data_ptr(), c.data_ptr()
        prog.launch(d, o, torch.cuda.current_stream(cuda))
        torch.cuda.synchronize()
        ref_v.append(v.cpu())
        ref_c.append(c.cpu().numpy().view(np.uint64))
    streams = [torch.cuda.current_stream(cuda), torch.cuda.Stream(cuda)]
    sdescs = []
    for si in range(2):
        row = []
        for d in descs:
            d2 = type(d).from_buffer_copy(d)
            if own_ws:
                wb = prog.workspace_bytes(d, 0)
                ws = torch.zeros(max(wb, 1), dtype=torch.uint8, device=cuda)
                keep.append(ws)
                d2.workspace, d2.workspace_bytes = ws.data_ptr(), wb
            row.append(d2)
        sdescs.append(row)
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    steps = 12
    verd = [torch.empty(n, dtype=torch.uint8, device=cuda) for _ in range(steps)]
    ev0 = torch.cuda.Event()
    ev0.record(streams[0])
    streams[1].wait_event(ev0)
    for i in range(steps):
        si = i % 2
        o = _lib.BatchOut()
        o.verdict, o.counters = verd[i].data_ptr(), cnt.data_ptr()
        prog.launch(sdescs[si][i % 3], o, streams[si])
    torch.cuda.synchronize()
    want = np.zeros(8, dtype=np.uint64)
    for i in range(steps):
        assert torch.equal(verd[i].cpu(), ref_v[i % 3]), (config, own_ws, i)
        want += ref_c[i % 3]
    assert list(cnt.cpu().numpy().view(np.uint64)) == list(want), (config, own_ws)
    prog.close()


def test_bench_line(cuda):
    """bench.py's contract line (two streams, the default) on a small run: one JSON line with the
    driver's keys, the roofline and its stream fields, and counters that add up to the packets."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "6", "--warmup",
                        "2", "--cpu-seconds", "0", "--packets", str(1 << 16), "--pool-mib", "8"],
                       capture_output=True, text=True, timeout=170, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["steps"] == 6 and d["n_gpus"] == 1 and d["config"]["streams"] == 2
    ro = d["roofline"]
    assert ro["streams"] == 2 and ro["kernel_avg_us"] > 0 and ro["kernel_single_us"] > 0
    c = d["counters"]
    assert c["drop"] + c["pass"] + c["other"] + c["faults"] <= 6 * (1 << 16)


@pytest.mark.parametrize("extra,env", [
    ([], {}),
    # two ranks on this one GPU through bench.py's own launcher (gloo: RCCL refuses two ranks on
    # one device): spawn, rendezvous, counter reduction, max over ranks, per-rank chunk pins
    (["--gpus", "2"], {"EBPFEMU_BENCH_BACKEND": "gloo"}),
    (["--config", "xdp", "--layout", "offsets"], {}),
])
def test_bench_line_pinned(cuda, extra, env):
    """The default weak-scaling line at full batch size (1 Mi packets, the pool of 8 chunks per
    rank) pins its timed counters to the oracle's fixture (tests/golden/bench_pins.json)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, **env)
    e.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "11",
                        "--warmup", "2", "--cpu-seconds", "0"] + extra,
                       capture_output=True, text=True, timeout=170, cwd=root, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    n = 2 if "--gpus" in extra else 1
    assert d["n_gpus"] == n and d["config"]["pool_batches"] == 8
    assert d["parity_pinned"] and f"k*{n}+r" in d["parity_pinned"], d.get("pin_note")
    c = d["counters"]
    assert c["drop"] + c["pass"] + c["other"] + c["faults"] == 11 * n * (1 << 20)


@pytest.mark.parametrize("slot,shift", [(64, 0), (80, 3), (80, 8), (81, 5)])
@pytest.mark.parametrize("name", ["5tuple", "5tuple_stack", "5tuple_xdp", "acl"])
def test_var_kernel_full_size_shuffled(cuda, name, slot, shift):
    """The compiled var kernels at full size (1 Mi packets: several tiles per persistent wave, so
    each tile's offsets and lengths arrive by the previous tile's metadata prefetch). The fixed
    5-tuple fixture's frames, stored `slot` bytes apart at `shift` (3, 8: every packet misaligned
    by the same amount -- 8 is a pcap capture's record layout -- so the var tile loop DMAs from
    16-byte aligned sources and realigns with one shift per tile; slot 81: a different
    misalignment per packet, the realign's per-lane select network) and listed in a shuffled
    order through offsets + lens: verdict, r0 and status i
    equal the fixed-slot kernel's for frame perm[i] (for the 5-tuple: the fixture's CRC and
    counters; the others run on fixed slots against the oracle in their own tests). Programs: the
    5-tuple, its stack-window form (ebpf_tile_jit_var_stack), the standard-XDP form over xdp_md
    contexts (the ctx synthesised in the window), the 97-instruction ACL."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    with open(os.path.join(GOLDEN, "workloads.json")) as f:
        g = json.load(f)["5tuple"]
    n = g["n"]
    buf = W.frames_fixed(n, 64, g["config_id"])
    prog = Program(W.program(name))
    xdp = name == "5tuple_xdp"
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    ref = prog.run(torch.from_numpy(buf).to(cuda), n=n, stride=64, counters=cnt, r0=True,
                   status=True, xdp_md=xdp)
    torch.cuda.synchronize()
    vref = ref.verdict.cpu().numpy()
    if name != "acl":  # the same verdicts as the 5-tuple's fixture (other instruction counts)
        assert zlib.crc32(vref.tobytes()) == g["verdict_crc32"]
        got = [int(x) for x in cnt.cpu().numpy().view(np.uint64)]
        assert got[:7] == g["counters"][:7]
        assert name != "5tuple" or got == g["counters"]

    big = np.zeros((n, slot), dtype=np.uint8)
    big[:, shift:shift + 64] = buf.reshape(n, 64)
    perm = np.random.default_rng(slot).permutation(n)
    offs = (perm.astype(np.int64) * slot + shift).astype(np.uint32)
    frames = torch.from_numpy(big.reshape(-1)).to(cuda)
    kw = dict(n=n, offsets=torch.from_numpy(offs.view(np.int32)).to(cuda),
              lens=torch.from_numpy(np.full(n, 64, dtype=np.int16)).to(cuda), xdp_md=xdp)
    # (offsets + lens: the var tile loop, ebpf_tile_jit_varl; stack-window programs the var kernel)
    want = _lib.EBPF_KERNEL_JIT_VARL_STACK if name == "5tuple_stack" else _lib.EBPF_KERNEL_JIT_VARL
    assert prog.batch_kernel(prog.make_batch(frames, **kw)) == want
    cnt2 = torch.zeros(8, dtype=torch.int64, device=cuda)
    res = prog.run(frames, counters=cnt2, r0=True, status=True, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(res.verdict.cpu().numpy(), vref[perm])
    assert np.array_equal(res.r0.cpu().numpy(), ref.r0.cpu().numpy()[perm])
    assert np.array_equal(res.status.cpu().numpy(), ref.status.cpu().numpy()[perm])
    assert torch.equal(cnt2, cnt)
    # the production outputs alone (verdicts + counters, liveness-pruned init)
    res = prog.run(frames, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(res.verdict.cpu().numpy(), vref[perm])
