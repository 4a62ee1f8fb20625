"""Programs past the compiler's near-branch reach (jit.cpp far mode; kJitMaxUops = 4096 micro-ops):
the reference runs programs of any length through one step() (emu.rs:452-458), so a 1000-
instruction parser must not drop from the compiled kernels to the general interpreter.

Far mode (compile_into_template, when a statement's body passes kFarLines): every body sits out
of line behind its kernel's code, entered and left by long jumps (s_getpc / s_setpc), its
out-of-line paths in islands between blocks, its long structural branches (the fast copy's
skip, a loop program's step-budget restart) as long jumps.

CPU: long forward, loop, stack-window and store-mode programs compile and assemble, in far mode
exactly when they are long (the benchmark programs never are). GPU: every output of the compiled
kernels == the general interpreter's (EBPF_BATCH_NO_JIT) == the oracle's, on the fixed-slot,
offsets + lens and init_regs layouts, with the route asserted (a compiled kernel, not the
interpreter)."""
import random

import pytest

from fuzzgen import gen_long_program, gen_packet

FAR = "; the program's code: out of line"


def _far(text: str) -> bool:
    return FAR in text


def test_benchmark_programs_not_far():
    """The benchmark programs compile as before (bodies inline, no long jumps)."""
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    for name in W.PROGRAMS:
        p = Program(W.program(name))
        assert p.compile(), name
        for v in (0, 1, 2):
            try:
                text = p.jit_asm(v)
            except Exception:
                continue
            assert not _far(text), (name, v)
        p.close()


@pytest.mark.parametrize("n", [400, 1200, 3000])
def test_long_forward_programs_compile(n):
    from ebpf_emu import Program

    rng = random.Random(n)
    for _ in range(2):
        p = Program(gen_long_program(rng, n))
        assert p.tier == 0 and p.forward_only and p.compile()
        for v in (0, 1, 2):
            text = p.jit_asm(v)
            if n >= 1200 or v == 2:  # (2: the block and exact copies)
                assert _far(text), (n, v)
            assert "s_setpc_b64 s[60:61]" in text or not _far(text)
        p.close()


def test_long_loop_programs_compile():
    from ebpf_emu import Program

    rng = random.Random(77)
    for n in (600, 2500):
        p = Program(gen_long_program(rng, n, loops=True))
        assert p.tier == 0 and not p.forward_only and p.compile()
        assert _far(p.jit_asm(2))
        with pytest.raises(Exception):  # (no forward variants for a loop program)
            p.jit_asm(1)
        p.close()


def test_long_stack_and_store_programs_compile():
    from ebpf_emu import Program

    rng = random.Random(78)
    for gen in (lambda: gen_long_program(rng, 1500, stack=True),
                lambda: gen_long_program(rng, 1500, store=True)):
        p = Program(gen())
        assert p.compile()
        assert _far(p.jit_asm(1))
        p.close()


def test_past_the_limit_interpreted():
    """Past kJitMaxUops the program loads and runs on the general interpreter (not compiled), and
    ebpf_prog_jit_error says so; a compiled program has no error."""
    from ebpf_emu import Program
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    p = Program(gen_long_program(random.Random(5), 4200))
    assert not p.compile()
    assert "past EBPF_MAX_COMPILED_UOPS (4096)" in p.jit_error, p.jit_error
    p.close()
    p = Program(W.program("acl_rules"))
    assert p.compile() and p.jit_error == ""
    p.close()
    # (a store at a constant address past the header window: the general interpreter's tier 1)
    p = Program(assemble("mov r3, 100\nstxw [r3+0], r3\nmov r0, 2\nexit"))
    assert not p.compile() and "tier 1" in p.jit_error, p.jit_error
    p.close()


def test_acl_rules_pins(oracle_mod):
    """bench.py --config acl_rules: the committed pins are this program's (its source is generated:
    workloads.acl_rules_source) and chunk 0's counters are the oracle's on dist.chunk_frames(0)."""
    import json
    import os

    from ebpf_emu import dist as D
    from ebpf_emu import workloads as W

    with open(os.path.join(os.path.dirname(__file__), "golden", "bench_pins.json")) as f:
        pin = json.load(f)["programs"]["acl_rules"]
    img = W.program("acl_rules")
    assert pin["program"] == img.hex() and len(img) // 8 == 1013
    _, _, cnt = oracle_mod.Program(img).run_batch(D.chunk_frames(0, D.CHUNK), D.CHUNK, stride=64,
                                                  mem_size=1024, r10=512, threads=4)
    assert [int(x) for x in cnt] == pin["chunk_counters"][0]
    assert 0.1 < cnt[1] / D.CHUNK < 0.4 and cnt[7] / D.CHUNK > 250  # (drops; steps per packet)


# ---------------------------------------------------------------------------------------------
def _kernel(img, dev, layout, pkts):
    import torch

    from ebpf_emu import Program, _lib
    from test_gpu_parity import _stage

    q = Program(img)
    q.compile()
    if layout == "fixed":
        fr = torch.zeros(64 * len(pkts), dtype=torch.uint8, device=dev)
        b = q.make_batch(fr, n=len(pkts), stride=64, max_steps=20000)
    else:
        fr, kw = _stage(pkts, dev, offsets_layout=True)
        b = q.make_batch(fr, max_steps=20000, **kw)
    k = q.batch_kernel(b)
    q.close()
    return _lib.KERNEL_NAMES[k]


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed", "offsets", "init_regs"])
@pytest.mark.parametrize("n", [500, 1500, 3500])
def test_long_forward_programs_vs_oracle(cuda, oracle_mod, layout, n):
    from test_gpu_jit import _run, _same, _vs_oracle

    rng = random.Random(1000 * n + ["fixed", "offsets", "init_regs"].index(layout))
    for it in range(2):
        img = gen_long_program(rng, n)
        kw, ir = {}, None
        if layout == "fixed":
            pkts = [bytes(rng.getrandbits(8) for _ in range(64)) for _ in range(rng.choice([64, 130]))]
            kw = dict(fixed_stride=64)
        else:
            pkts = [gen_packet(rng) for _ in range(rng.choice([64, 100]))]
            kw = dict(offsets_layout=True)
            if layout == "init_regs":
                ir = [rng.getrandbits(64) if rng.random() < 0.5 else rng.randrange(0, 200)
                      for _ in range(11)]
                ir[1] = 0
                kw["init_regs"] = ir
        name = _kernel(img, cuda, "fixed" if layout == "fixed" else "offsets", pkts)
        assert name.startswith("ebpf_tile_jit"), name
        got = _run(img, pkts, cuda, **kw)
        ref = _run(img, pkts, cuda, no_jit=True, **kw)
        _same(got, ref, f"{layout} n {n} it {it}")
        _vs_oracle(oracle_mod, img, pkts, got, init_regs=ir, tag=f"{layout} {n} {it}")
        prod = _run(img, pkts, cuda, prod=True, **kw)
        _same(prod, got, f"prod {layout} n {n} it {it}", keys=("status", "r0", "verdict", "counters"))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [700, 2500])
def test_long_loop_programs_vs_oracle(cuda, oracle_mod, n):
    """Counted loops inside a long program: the compiled loop kernel in far mode (its step-budget
    restart a long jump), including a budget that binds (the exact copy)."""
    from test_gpu_jit import _run, _same, _vs_oracle

    rng = random.Random(n)
    for it in range(2):
        img = gen_long_program(rng, n, loops=True)
        pkts = [gen_packet(rng) for _ in range(rng.choice([64, 100]))]
        name = _kernel(img, cuda, "offsets", pkts)
        assert name.startswith("ebpf_tile_jit_loop"), name
        got = _run(img, pkts, cuda, offsets_layout=True)
        ref = _run(img, pkts, cuda, offsets_layout=True, no_jit=True)
        _same(got, ref, f"loop n {n} it {it}")
        _vs_oracle(oracle_mod, img, pkts, got, tag=f"loop {n} {it}")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["stack", "store"])
def test_long_stack_and_store_programs_vs_oracle(cuda, oracle_mod, kind):
    """A stack-window program (fixed slots: ebpf_tile_jit_stack) and a store-mode program (offsets
    + lens: the var tile loop's stack statement, its deopt list re-run) of 1500 instructions."""
    # (gen_long_program's stack and store forms: gen_stack_program's constant-address loads
    # around r10 - k keep a long program's batches off the stack kernel (host.cpp
    # stack_launch_ok), and gen_store_program's early exits leave a long program a short one)
    from test_gpu_jit import _run, _same, _vs_oracle

    rng = random.Random(31 if kind == "stack" else 32)
    for it in range(2):
        if kind == "stack":
            img = gen_long_program(rng, 1500, stack=True)
            pkts = [bytes(rng.getrandbits(8) for _ in range(64)) for _ in range(130)]
            kw = dict(fixed_stride=64)
        else:
            img = gen_long_program(rng, 1500, store=True)
            pkts = [gen_packet(rng, 100) for _ in range(130)]
            kw = dict(offsets_layout=True)
        name = _kernel(img, cuda, "fixed" if kind == "stack" else "offsets", pkts)
        assert name.startswith("ebpf_tile_jit"), name
        got = _run(img, pkts, cuda, prod=True, **kw)
        ref = _run(img, pkts, cuda, prod=True, no_jit=True, **kw)
        _same(got, ref, f"{kind} it {it}", keys=("status", "r0", "verdict", "counters"))
        full = _run(img, pkts, cuda, **kw)
        _vs_oracle(oracle_mod, img, pkts, full, tag=f"{kind} {it}")


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed", "offsets"])
def test_long_programs_xdp_md(cuda, oracle_mod, layout):
    """Far-mode code on xdp_md batches (the ctx synthesised in the window, xdp.rs:16-20): the
    production outputs and the counters == the oracle's, every output == the general
    interpreter's, on a compiled kernel."""
    import numpy as np
    import torch

    from ebpf_emu import Program, _lib
    from test_gpu_parity import _stage

    rng = random.Random(91 + (layout == "offsets"))
    for it in range(2):
        img = gen_long_program(rng, 1200)
        prog = Program(img)
        assert prog.compile()
        if layout == "fixed":
            n = 300
            buf = np.frombuffer(bytes(rng.getrandbits(8) for _ in range(64 * n)), dtype=np.uint8)
            frames = torch.from_numpy(buf.copy()).to(cuda)
            kw = dict(n=n, stride=64)
            okw = dict(stride=64)
        else:
            pkts = [gen_packet(rng, 100) for _ in range(300)]
            frames, kw = _stage(pkts, cuda, offsets_layout=True)
            n = len(pkts)
            buf = frames.cpu().numpy()
            okw = dict(offsets=kw["offsets"].cpu().numpy().view(np.uint32),
                       lens=kw["lens"].cpu().numpy().view(np.uint16))
        k = prog.batch_kernel(prog.make_batch(frames, xdp_md=True, mem_size=1024, **kw))
        assert _lib.KERNEL_NAMES[k].startswith("ebpf_tile_jit"), _lib.KERNEL_NAMES[k]
        cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
        v = prog.run(frames, mem_size=1024, counters=cnt, xdp_md=True, **kw)
        rs = prog.run(frames, mem_size=1024, verdict=False, r0=True, status=True, xdp_md=True, **kw)
        full = prog.run(frames, mem_size=1024, r0=True, status=True, regs=True, xdp_md=True, **kw)
        gen = prog.run(frames, mem_size=1024, r0=True, status=True, regs=True, xdp_md=True,
                       generic=True, **kw)
        torch.cuda.synchronize()
        r0, st, ocnt = oracle_mod.Program(img).run_batch(buf, n, mem_size=1024, xdp_md=True,
                                                         threads=4, **okw)
        assert np.array_equal(rs.status.cpu().numpy(), st), it
        ok = st == 0
        assert np.array_equal(rs.r0.cpu().numpy().view(np.uint64)[ok], r0[ok]), it
        want_v = np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8)
        assert np.array_equal(v.verdict.cpu().numpy(), want_v), it
        assert list(cnt.cpu().numpy().view(np.uint64)) == list(ocnt), it
        for key in ("r0", "status", "regs"):
            assert torch.equal(getattr(full, key), getattr(gen, key)), (it, key)
        prog.close()


@pytest.mark.gpu
def test_long_programs_fuzz(cuda, oracle_mod):
    """Random long programs of every form (forward, counted loops, stack window, packet-pointer
    stores; 400-2500 instructions) on offsets + lens batches: production outputs and counters ==
    the oracle's, every output == the general interpreter's, and each on a compiled kernel."""
    from test_gpu_jit import _run, _same, _vs_oracle

    rng = random.Random(20261018)
    for it in range(12):
        kind = ["fwd", "loop", "stack", "store"][it % 4]
        n = rng.choice([400, 900, 1600, 2500])
        img = gen_long_program(rng, n, loops=kind == "loop", stack=kind == "stack",
                               store=kind == "store")
        pkts = [gen_packet(rng, 100) for _ in range(rng.choice([64, 130]))]
        name = _kernel(img, cuda, "offsets", pkts)
        assert name.startswith("ebpf_tile_jit"), (kind, n, name)
        prod = _run(img, pkts, cuda, prod=True, offsets_layout=True)
        ref = _run(img, pkts, cuda, prod=True, no_jit=True, offsets_layout=True)
        _same(prod, ref, f"{kind} {n} it {it}", keys=("status", "r0", "verdict", "counters"))
        full = _run(img, pkts, cuda, offsets_layout=True)
        _vs_oracle(oracle_mod, img, pkts, full, tag=f"{kind} {n} {it}")
