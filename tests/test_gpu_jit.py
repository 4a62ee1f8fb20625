"""The program compiler (csrc/jit.cpp): forward-only tier-0 programs of <= 256 micro-ops compiled
to gfx950 code for the tile kernel, instead of interpreted (tile_kernel up to 62, dag_kernel
beyond).

CPU (no GPU needed, the compiler and assembler run in process): every such program compiles,
the assembler accepts it, and its code has no interpreter machinery left (no index mode, no
dispatch jumps, no micro-op loads).

GPU: the compiled kernels against the oracle and against the tile interpreter on the same batch
(EBPF_BATCH_NO_JIT) -- every output bit-identical, counters included -- in the fixed-slot layout
(ebpf_tile_jit_fixed), the offsets + lens layout (ebpf_tile_jit_var) and with init_regs (the
variant whose constant-address loads stay register-based)."""
import random

import numpy as np
import pytest

from fuzzgen import gen_packet, gen_program

STEPS = 20000


def _eligible(img):
    from ebpf_emu import Program

    p = Program(img)
    try:
        return p, p.compile()
    except Exception:
        p.close()
        raise


def test_workloads_compile():
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    for name, src in W.PROGRAMS.items():
        p, ok = _eligible(assemble(src))
        if name == "mac_swap_tx":  # packet-window stores + a stack atomic: memory tier 0.5
            assert p.tier == 1 and p.stack_window == 8
        assert ok, name
        # forward-only programs: the forward kernels (0, 1) and the loop kernel (2, for budgets
        # that can bind); the checksum loops: the loop kernel only
        # (the stack programs: the main.rs layout's forward kernels, and the loop kernel's stack
        # variant unless they store into the packet; the ACL, past 62 micro-ops: the forward
        # kernels only, budgets that bind run dag_kernel / interp_kernel)
        # (the NAT rewrite and the responder store through a register: store mode, variant 1 only)
        variants = ((2,) if name in ("checksum", "checksum_stack", "checksum_xdp",
                                     "checksum_xdp_reload")
                    else (1,) if name in ("mac_swap_tx", "nat", "responder")
                    else (1, 2) if name == "5tuple_stack" else (0, 1) if name == "acl"
                    else (0, 1, 2))
        for variant in variants:
            text = p.jit_asm(variant)
            key = "; compiled eBPF loop program" if variant == 2 else "; compiled eBPF program"
            body = text[text.index(key):]
            body = body[:body.index(".Ldone")]
            for word in ("s_set_gpr_idx", "s_setpc", "s_load_dwordx16", "s_ff1"):
                assert word not in body, (name, word)
        if name in ("checksum", "checksum_stack"):
            with pytest.raises(Exception):
                p.jit_asm(1)
        if name == "checksum_xdp":  # the xdp_md copies: the ctx known (5), rebased in place (6)
            assert "v_add_u32 v4, 8, v31" not in p.jit_asm(5)
            assert "v_add_u32 v4, 8, v31" in p.jit_asm(6)
        p.close()


def test_xdp_loop_rebase_eligibility():
    """Variant 6 (xdp_md loop programs in place, jit.cpp Compiler::xdp_rebase) is compiled only
    when the range analysis proves every packet load past the ctx: the byte sum, the bound
    reloaded from the ctx (through r1 or a saved copy of it), word + half loads behind a pointer
    compared with data_end; not a
    program whose ctx-shaped load may read the ctx, nor a load at a fixed offset below 8."""
    import test_gpu_xdp_md as X
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    for src, rebased in ((X.XDP_SUM, True), (X.XDP_SUM_RELOAD, True), (X.XDP_SUM_WIDE, True),
                         (X.XDP_SUM_CTX_SAVED, True), (X.XDP_R1_MOVED, False),
                         # (a copy of r1 overwritten before its ctx-shaped load: not the ctx)
                         (X.XDP_SUM_CTX_SAVED.replace("mov r0, 0", "mov r0, 0\n    add r7, 1"),
                          False),
                         (X.XDP_SUM.replace("mov r0, 0", "ldxb r0, [r1+2]"), False)):
        p = Program(assemble(src))
        assert p.compile()
        p.jit_asm(5)
        if rebased:
            text = p.jit_asm(6)
            assert "v_add_u32 v4, 8, v31" in text  # (r2 = 8 + LEN)
        else:
            with pytest.raises(Exception):
                p.jit_asm(6)
        p.close()


def test_fuzz_programs_compile():
    """Random forward-only tier-0 programs: each compiles and assembles (a template or
    token-expansion bug is an assembler error here, on the CPU)."""
    rng = random.Random(31337)
    n = 0
    for _ in range(300):
        img = gen_program(rng, allow_loops=False, tier0=True)
        try:
            p, ok = _eligible(img)
        except Exception as e:  # decode errors: not a program
            assert "ebpf_prog_load" in str(e) or "decode" in str(e).lower(), e
            continue
        if ok:
            n += 1
            assert p.jit_asm(2)
            if p.forward_only:
                assert p.jit_asm(0) and p.jit_asm(1)
        p.close()
    assert n >= 150


def test_fuzz_loop_programs_compile():
    """Random tier-0 programs with back edges: the loop kernel compiles and assembles."""
    rng = random.Random(4711)
    n = 0
    for _ in range(200):
        img = gen_program(rng, allow_loops=True, tier0=True)
        try:
            p, ok = _eligible(img)
        except Exception as e:
            assert "ebpf_prog_load" in str(e) or "decode" in str(e).lower(), e
            continue
        if ok:
            n += 1
            assert p.jit_asm(2)
        p.close()
    assert n >= 100


def test_loop_range_proofs_compile():
    """The loop compiler's range analysis (jit.cpp prove_loads) proves exactly the byte scans whose
    index is non-negative and below r2 on every path (test_gpu_loops.RANGE_PROGRAMS); the proven
    copy has no bounds check on those loads. Random scans compile either way."""
    import random as _r

    from ebpf_emu import Program
    from ebpf_emu.asm import assemble
    from test_gpu_loops import RANGE_PROGRAMS, gen_scan_program

    for name, src in RANGE_PROGRAMS.items():
        p = Program(assemble(src))
        assert p.compile()
        text = p.jit_asm(2)
        assert ("one-byte loads proven in bounds" in text) == name.startswith("proven"), name
        p.close()
    from test_gpu_loops import COUNTED_EDGE_PROGRAMS

    for name, src in COUNTED_EDGE_PROGRAMS.items():  # (their GPU runs: test_counted_loop_edges)
        p = Program(assemble(src))
        assert p.compile()
        assert "counted loop" in p.jit_asm(2), name
        p.close()
    rng = _r.Random(3)
    proven = 0
    for _ in range(60):
        p = Program(assemble(gen_scan_program(rng)))
        assert p.compile()
        proven += "one-byte loads proven in bounds" in p.jit_asm(2)
        p.close()
    assert 6 <= proven <= 54, proven


def test_xdp_ctx_data_folded():
    """xdp_md batches get a compiled variant of their own (host.cpp fold_const_loads xdp) where a
    standard XDP program's ctx->data load is the constant 8 and the packet loads through it are
    constant-address loads; programs that gain nothing from it get none."""
    from ebpf_emu import Program
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble
    from test_gpu_xdp_md import XDP_CTX_MIX, XDP_PARSE

    def body(text):
        b = text[text.index("; JIT N=0"):]
        b = b[b.index("; compiled eBPF program"):]
        return b[:b.index(".Ldone")].count("\n")

    for img in (W.program("5tuple_xdp"), assemble(XDP_PARSE)):
        p = Program(img)
        assert p.compile()
        assert body(p.jit_asm(3)) < body(p.jit_asm(1))
        p.close()
    for img in (W.program("5tuple"), assemble(XDP_CTX_MIX)):
        p = Program(img)
        assert p.compile()
        with pytest.raises(Exception):
            p.jit_asm(3)
        p.close()


# ---------------------------------------------------------------------------------------------
_PROG = {}  # the last program _run loaded (the compiled, the no-JIT and the production runs of
# one image share it: one load and module upload instead of three)


def _prog(img):
    from ebpf_emu import Program

    if img not in _PROG:
        for q in _PROG.values():
            q.close()
        _PROG.clear()
        q = Program(img)
        assert q.compile()
        _PROG[img] = q
    return _PROG[img]


def _run(img, pkts, dev, fixed_stride=None, offsets_layout=False, init_regs=None, no_jit=False,
         mem_size=1024, r10=512, prod=False):
    """prod: the production outputs only -- a verdict + counters launch (k_flags = 0) and an r0 +
    status launch, neither asking for registers, so the compiled kernels run their liveness-pruned
    register init (;@@JITINIT@@, jit.cpp live_in) instead of initialising every register."""
    import torch

    from test_gpu_parity import _stage

    prog = _prog(img)
    if fixed_stride:  # no lens: every packet is `fixed_stride` bytes (the fixed-slot layout)
        buf = np.zeros(len(pkts) * fixed_stride, dtype=np.uint8)
        for i, p in enumerate(pkts):
            assert len(p) == fixed_stride
            buf[i * fixed_stride:(i + 1) * fixed_stride] = np.frombuffer(p, dtype=np.uint8)
        frames = torch.tensor(buf, device=dev)
        kw = dict(n=len(pkts), stride=fixed_stride)
    else:
        frames, kw = _stage(pkts, dev, offsets_layout=offsets_layout)
    ir = None
    if init_regs is not None:
        ir = torch.tensor(np.array(init_regs, dtype=np.uint64).view(np.int64), device=dev)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    if prod:
        v = prog.run(frames, mem_size=mem_size, r10=r10, max_steps=STEPS, verdict=True,
                     counters=cnt, init_regs=ir, no_jit=no_jit, **kw)
        rs = prog.run(frames, mem_size=mem_size, r10=r10, max_steps=STEPS, verdict=False, r0=True,
                      status=True, init_regs=ir, no_jit=no_jit, **kw)
        torch.cuda.synchronize()
        out = dict(status=rs.status.cpu().numpy(), r0=rs.r0.cpu().numpy().view(np.uint64),
                   verdict=v.verdict.cpu().numpy(), counters=cnt.cpu().numpy().view(np.uint64))
        return out
    res = prog.run(frames, mem_size=mem_size, r10=r10, max_steps=STEPS, verdict=True, r0=True,
                   status=True, regs=True, counters=cnt, init_regs=ir, no_jit=no_jit, **kw)
    torch.cuda.synchronize()
    out = dict(status=res.status.cpu().numpy(), r0=res.r0.cpu().numpy().view(np.uint64),
               verdict=res.verdict.cpu().numpy(), regs=res.regs.cpu().numpy().view(np.uint64),
               counters=cnt.cpu().numpy().view(np.uint64))
    return out


def _vs_oracle(oracle_mod, img, pkts, got, init_regs=None, tag=""):
    op = oracle_mod.Program(img)
    cnt = np.zeros(8, dtype=np.uint64)
    for i, p in enumerate(pkts):
        if init_regs is None:
            st, regs, _mem, steps = op.run_full(p, 1024, 512, STEPS)
        else:
            st, regs, _mem, steps = op.run_full(p, 1024, 512, STEPS, init_regs=list(init_regs))
        ctx = f"{tag} pkt {i} prog {img.hex()} pkt {p.hex()}"
        assert got["status"][i] == st, ctx
        if st == 0:
            assert [int(v) for v in got["regs"][i]] == regs, ctx
            cnt[regs[0] if regs[0] < 5 else 5] += 1
        else:
            cnt[6] += 1
        cnt[7] += steps
    assert list(got["counters"]) == list(cnt), tag


def _same(a, b, ctx, keys=("status", "r0", "verdict", "regs", "counters")):
    for k in keys:
        assert np.array_equal(a[k], b[k]), f"{ctx}: {k} differs"


def test_fuzz_large_programs_compile():
    """Forward-only tier-0 programs of 63-256 micro-ops (past the tile interpreter's 62) compile
    too, with parked pcs above the inline-constant range staged through SGPRs."""
    rng = random.Random(4711)
    n = 0
    for _ in range(60):
        img = gen_program(rng, n=rng.randrange(70, 250), allow_loops=False, tier0=True)
        try:
            p, ok = _eligible(img)
        except Exception as e:
            assert "ebpf_prog_load" in str(e) or "decode" in str(e).lower(), e
            continue
        if p.forward_only and ok:
            n += 1
            assert p.jit_asm(0) and p.jit_asm(1)
        p.close()
    assert n >= 20


def test_fuzz_large_loop_programs_compile():
    """Tier-0 programs with back edges of 63-256 micro-ops: the loop program compiler takes them
    (both copies and the exact-budget copy), with back-edge selects of pcs above 64."""
    rng = random.Random(4712)
    n = 0
    for _ in range(60):
        img = gen_program(rng, n=rng.randrange(70, 250), allow_loops=True, tier0=True)
        try:
            p, ok = _eligible(img)
        except Exception as e:
            assert "ebpf_prog_load" in str(e) or "decode" in str(e).lower(), e
            continue
        if p.tier == 0:
            assert ok
            assert p.jit_asm(2)
            n += 1
        p.close()
    assert n >= 20


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed", "offsets", "init_regs"])
@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("size", ["small", "large"])
def test_compiled_vs_interpreter_and_oracle(cuda, oracle_mod, layout, seed, size):
    """size large: 63-256 micro-ops, compiled instead of dag_kernel (the no-JIT reference)."""
    rng = random.Random(5150 + 7 * seed + 1000 * ["fixed", "offsets", "init_regs"].index(layout) +
                        (0 if size == "small" else 99991))
    n_run = 0
    for it in range(40 if size == "small" else 16):
        img = gen_program(rng, allow_loops=False, tier0=True,
                          n=None if size == "small" else rng.randrange(70, 250))
        try:
            oracle_mod.Program(img)
            p, ok = _eligible(img)
            p.close()
        except Exception:
            continue
        if not ok:
            continue
        if size == "large":  # compiled, not dag_kernel
            import torch

            from ebpf_emu import Program, _lib
            q = Program(img)
            q.compile()
            fr = torch.zeros(64 * 64, dtype=torch.uint8, device=cuda)
            k = q.batch_kernel(q.make_batch(fr, n=64, stride=64, max_steps=STEPS))
            q.close()
            assert k in (_lib.EBPF_KERNEL_JIT_FIXED, _lib.EBPF_KERNEL_JIT_FIXED_OCC), _lib.KERNEL_NAMES[k]
        kw = {}
        ir = None
        if layout == "fixed":
            stride = rng.choice([64, 128])
            pkts = [bytes(rng.getrandbits(8) for _ in range(stride))
                    for _ in range(rng.choice([64, 100, 130]))]
            kw = dict(fixed_stride=stride)
        else:
            pkts = [gen_packet(rng) for _ in range(rng.choice([64, 65, 100, 130]))]
            kw = dict(offsets_layout=True)
            if layout == "init_regs":
                ir = [rng.getrandbits(64) if rng.random() < 0.5 else rng.randrange(0, 200)
                      for _ in range(11)]
                ir[1] = 0  # r1 = the image address, so the loads stay mostly in bounds
                kw["init_regs"] = ir
        got = _run(img, pkts, cuda, **kw)
        ref = _run(img, pkts, cuda, no_jit=True, **kw)
        _same(got, ref, f"{layout} seed {seed} it {it} prog {img.hex()}")
        _vs_oracle(oracle_mod, img, pkts, got, init_regs=ir, tag=f"{layout} {seed} {it}")
        # the production path (no registers asked for): the same results as the full-output run
        prod = _run(img, pkts, cuda, prod=True, **kw)
        _same(prod, got, f"prod {layout} seed {seed} it {it} prog {img.hex()}",
              keys=("status", "r0", "verdict", "counters"))
        n_run += 1
    assert n_run >= (20 if size == "small" else 6)


@pytest.mark.gpu
def test_compiled_fixed_small_image(cuda, oracle_mod):
    """Fixed-slot batches whose image is as small as the slots (mem_size = stride = 64): window
    loads past the image fault (ST_MEM / ST_MEM_UB), so the compiled kernel takes its checked copy
    of the program instead of the preloaded-window one. Both against the interpreter and the
    oracle."""
    from ebpf_emu.asm import assemble

    srcs = ["ldxdw r0, [r1+60]\nexit", "ldxw r0, [r1+62]\nexit", "ldxb r0, [r1+63]\nexit",
            "ldxh r3, [r1+12]\nldxdw r0, [r1+58]\nadd r0, r3\nexit",
            "mov r0, 2\njlt r2, 70, +1\nldxdw r0, [r1+60]\nexit"]
    rng = random.Random(99)
    pkts = [bytes(rng.getrandbits(8) for _ in range(64)) for _ in range(130)]
    for src in srcs:
        img = assemble(src)
        for mem in (64, 1024):
            got = _run(img, pkts, cuda, fixed_stride=64, mem_size=mem)
            ref = _run(img, pkts, cuda, fixed_stride=64, mem_size=mem, no_jit=True)
            _same(got, ref, f"{src!r} mem {mem}")
            op = oracle_mod.Program(img)
            for i, p in enumerate(pkts[:20]):
                st, regs, _m, _s = op.run_full(p, mem, 512, STEPS)
                assert got["status"][i] == st, (src, mem, i)
                if st == 0:
                    assert int(got["r0"][i]) == regs[0], (src, mem, i)


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["drop", "5tuple"])
def test_workloads_compiled_vs_interpreter(cuda, oracle_mod, config):
    """The bench workloads (BASELINE configs 1-4) on 8192 synthetic 64-byte frames, fixed-slot
    layout: compiled == interpreted == oracle."""
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    img = assemble(W.PROGRAMS[config])
    frames = W.frames_fixed(8192, 64)
    pkts = [bytes(frames[i * 64:(i + 1) * 64]) for i in range(8192)]
    got = _run(img, pkts, cuda, fixed_stride=64)
    ref = _run(img, pkts, cuda, fixed_stride=64, no_jit=True)
    _same(got, ref, config)
    sub = {k: v[:512] for k, v in got.items() if k != "counters"}
    sub["counters"] = _cnt(oracle_mod, img, pkts[:512])
    _vs_oracle(oracle_mod, img, pkts[:512], sub, tag=config)


def _cnt(oracle_mod, img, pkts):
    op = oracle_mod.Program(img)
    cnt = np.zeros(8, dtype=np.uint64)
    for p in pkts:
        st, regs, _mem, steps = op.run_full(p, 1024, 512, STEPS)
        if st == 0:
            cnt[regs[0] if regs[0] < 5 else 5] += 1
        else:
            cnt[6] += 1
        cnt[7] += steps
    return cnt


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["drop", "5tuple"])
def test_compiled_large_batches(cuda, config):
    """Batches of several tiles per wave for the compiled fixed-slot kernel (tiles handed out
    within each workgroup by its LDS counter, interp.hip tile_body) with ragged tails: three
    launches in a row on one workspace (counted counter shards reused) each equal the tile
    interpreter, verdicts and counters."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    prog = Program(assemble(W.PROGRAMS[config]))
    assert prog.compile()
    for n in (786432 + 64 * 5 + 7, 2500013):
        frames = torch.from_numpy(W.frames_fixed(n, 64, n % 7)).to(cuda)
        ref_cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
        ref = prog.run(frames, n=n, stride=64, counters=ref_cnt, no_jit=True)
        torch.cuda.synchronize()
        ref_v = ref.verdict.cpu().numpy()
        for rep in range(3):
            cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
            got = prog.run(frames, n=n, stride=64, counters=cnt)
            torch.cuda.synchronize()
            assert np.array_equal(got.verdict.cpu().numpy(), ref_v), (config, n, rep)
            assert cnt.cpu().tolist() == ref_cnt.cpu().tolist(), (config, n, rep)
            assert int(cnt[:7].sum()) == n
    prog.close()


@pytest.mark.gpu
def test_tile_loop_reentry(cuda, monkeypatch):
    """The compiled fixed-slot kernel's statement runs at most 511 tiles per entry before the
    C++ unpacks the packed counter buckets (interp.hip ebpf_tile_jit_fixed): with the grid capped
    to one workgroup (EBPFEMU_FIXED_WGS=1, read per launch: 16 waves), 600 Ki packets give each
    wave ~600 tiles. Verdicts and counters equal the tile interpreter's."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    n = 600 * 1024 + 13
    frames = torch.from_numpy(W.frames_fixed(n, 64, 9)).to(cuda)
    for name in ("5tuple", "drop"):
        prog = Program(assemble(W.PROGRAMS[name]))
        assert prog.compile()
        rc = torch.zeros(8, dtype=torch.int64, device=cuda)
        ref = prog.run(frames, n=n, stride=64, counters=rc, no_jit=True)
        monkeypatch.setenv("EBPFEMU_FIXED_WGS", "1")
        gc = torch.zeros(8, dtype=torch.int64, device=cuda)
        got = prog.run(frames, n=n, stride=64, counters=gc)
        torch.cuda.synchronize()
        monkeypatch.delenv("EBPFEMU_FIXED_WGS")
        assert np.array_equal(got.verdict.cpu().numpy(), ref.verdict.cpu().numpy()), name
        assert gc.cpu().tolist() == rc.cpu().tolist(), name
        assert int(gc[:7].sum()) == n
        prog.close()


