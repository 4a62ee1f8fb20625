"""CALL / EXIT off the general interpreter (host.cpp flatten_calls): a program with local calls
runs on the compiled kernels as one copy per reachable frame stack -- a CALL a jump into the
callee's copy, an EXIT with a non-empty stack a jump to the popped pc (emu.rs:265-279, Q12: the
pushed pc is the callee's entry + 1, no registers saved). Checked against the oracle (status,
r0, registers, retired steps) and the general interpreter's frame stack (EBPF_BATCH_GENERIC),
with binding step budgets; recursion flattens too while its 65 frame stacks x the recursive
body's pcs fit kJitMaxUops (ST_CALLDEPTH at 65 frames), else keeps the general interpreter."""
import random

import numpy as np
import pytest

from fuzzgen import gen_call_program, gen_packet
from test_gpu_parity import (_check_against_oracle, _check_prod_against_oracle, _run_full,
                             _run_prod, _same_outputs)

# f is called twice (a nested call, then from main); the callee runs from its entry, and the EXIT
# returns to entry + 1 (the reference's push of pc + 1 after the jump): f's body runs again there
NESTED = """
    mov r0, 1
    ldxb r3, [r1+0]
    call f
    add r0, 100
    call g
    add r0, 1000
    exit
f:
    add r0, r3
    lsh r0, 1
    exit
g:
    call f
    add r0, 7
    exit
"""

# unbounded recursion: every call jumps back to the program's start and pushes pc 1, so the
# stack grows to 64 frames and the 65th push faults ST_CALLDEPTH. 65 stacks x 2 pcs fit the
# compiled kernels (a forward-only program of 129 micro-ops), and so do RECURSE_BIG's 65 x 5 (325
# copies: past the 256 of rounds 1-4, inside kJitMaxUops = 4096); RECURSE_HUGE's 65 x 70 do not
# (the general interpreter's frame stack)
RECURSE = """
top:
    add r0, 1
    call top
    exit
"""
RECURSE_BIG = """
top:
    add r0, 1
    xor r0, r2
    lsh r0, 1
    add r0, r1
    call top
    exit
"""
RECURSE_HUGE = "top:\n" + "".join(f"    add r0, {k}\n    xor r0, r2\n" for k in range(34)) + """
    call top
    exit
"""


def test_flatten_compiles():
    """Programs with calls that do not recurse compile (the copies are an ordinary tier-0
    program); recursion does not flatten and keeps the general interpreter."""
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    p = Program(assemble(NESTED))
    assert p.forward_only and p.compile()
    p.close()
    p = Program(assemble(RECURSE))
    assert p.forward_only and p.compile()
    p.close()
    p = Program(assemble(RECURSE_BIG))
    assert p.forward_only and p.compile()
    p.close()
    p = Program(assemble(RECURSE_HUGE))
    assert not p.forward_only and not p.compile()
    p.close()
    rng = random.Random(5)
    flat = 0
    for _ in range(200):
        p = Program(gen_call_program(rng, loops=rng.random() < 0.3))
        flat += p.compile()
        p.close()
    assert flat >= 60, flat


@pytest.mark.gpu
def test_call_programs_directed(cuda, oracle_mod):
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu.asm import assemble

    rng = random.Random(1)
    pkts = [gen_packet(rng) for _ in range(130)]
    fwd = (_lib.EBPF_KERNEL_JIT_VAR, _lib.EBPF_KERNEL_JIT_VARL, _lib.EBPF_KERNEL_JIT_FIXED,
           _lib.EBPF_KERNEL_JIT_FIXED_OCC)
    for src, kern in ((NESTED, fwd), (RECURSE, fwd), (RECURSE_BIG, fwd),
                      (RECURSE_HUGE, (_lib.EBPF_KERNEL_GENERAL_T1,))):
        img = assemble(src)
        p = Program(img)
        frames = torch.zeros(64 * 64, dtype=torch.uint8, device=cuda)
        assert p.batch_kernel(p.make_batch(frames, n=64, stride=64)) in kern
        p.close()
        got = _run_full(img, pkts, cuda)
        _check_against_oracle(oracle_mod, img, pkts, got, tag=src[:20])
        _same_outputs(got, _run_full(img, pkts, cuda, generic=True), src[:20])
        prod = _run_prod(img, pkts, cuda)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, tag="prod " + src[:20])
    assert (got["status"] == 6).all()  # RECURSE_HUGE: ST_CALLDEPTH


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_fuzz_call_programs(cuda, oracle_mod, seed):
    """Random programs with calls (gen_call_program), forward-only and looping, with budgets that
    bind: the production outputs against the oracle, every output against the general
    interpreter's frame stack; most of them on the compiled kernels."""
    from ebpf_emu import Program, _lib

    import torch

    rng = random.Random(9090 + seed)
    routes = {}
    for it in range(30):
        img = gen_call_program(rng, loops=it % 3 == 0)
        steps = rng.choice([2000, 60])
        pkts = [gen_packet(rng) for _ in range(rng.choice([64, 100]))]
        layout = dict(offsets_layout=True, align=16) if it % 2 else dict()
        p = Program(img)
        frames = torch.zeros(64 * 64, dtype=torch.uint8, device=cuda)
        k = p.batch_kernel(p.make_batch(frames, n=64, stride=64, max_steps=steps))
        routes[_lib.KERNEL_NAMES[k]] = routes.get(_lib.KERNEL_NAMES[k], 0) + 1
        p.close()
        prod = _run_prod(img, pkts, cuda, max_steps=steps, **layout)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, max_steps=steps,
                                   tag=f"seed {seed} it {it} {img.hex()}")
        full = _run_full(img, pkts, cuda, max_steps=steps, **layout)
        gen = _run_full(img, pkts, cuda, max_steps=steps, generic=True, **layout)
        _same_outputs(full, gen, f"seed {seed} it {it} {img.hex()}")
    compiled = sum(v for k, v in routes.items() if "general" not in k.lower())
    assert compiled >= 10, routes


def test_call_workload_verdicts_cpu(oracle_mod):
    """workloads.FIVE_TUPLE_CALL (the L4 decision as a local function) returns the 5-tuple's
    verdicts in the oracle (its callee body is idempotent under the reference's entry + 1 return
    address), and flattens onto the compiled kernels."""
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    frames = W.frames_fixed(2048, 64)
    pkts = [bytes(frames[i * 64:(i + 1) * 64]) for i in range(2048)]
    a = oracle_mod.Program(W.program("5tuple_call"))
    b = oracle_mod.Program(W.program("5tuple"))
    for p in pkts:
        sa, ra, _m, _s = a.run_full(p, 1024, 512, 10000)
        sb, rb, _m, _s = b.run_full(p, 1024, 512, 10000)
        assert (sa, ra[0]) == (sb, rb[0])
    p = Program(W.program("5tuple_call"))
    assert p.forward_only and p.compile()
    p.close()


@pytest.mark.gpu
def test_call_workload(cuda, oracle_mod):
    """The bench's call workload on 8192 frames: routed to the compiled fixed-slot kernel,
    compiled == general interpreter (frame stack) == oracle."""
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from test_gpu_jit import _run, _same, _vs_oracle, _cnt

    img = W.program("5tuple_call")
    frames = W.frames_fixed(8192, 64)
    pkts = [bytes(frames[i * 64:(i + 1) * 64]) for i in range(8192)]
    p = Program(img)
    dev = torch.zeros(64 * 64, dtype=torch.uint8, device=cuda)
    assert p.batch_kernel(p.make_batch(dev, n=64, stride=64)) in (_lib.EBPF_KERNEL_JIT_FIXED,
                                                                  _lib.EBPF_KERNEL_JIT_FIXED_OCC)
    p.close()
    got = _run(img, pkts, cuda, fixed_stride=64)
    gen = _run_full(img, pkts[:1024], cuda, generic=True)
    assert (got["status"][:1024] == gen["status"]).all()
    assert (got["r0"][:1024] == gen["regs"][:, 0]).all()
    sub = {k: v[:512] for k, v in got.items() if k != "counters"}
    sub["counters"] = _cnt(oracle_mod, img, pkts[:512])
    _vs_oracle(oracle_mod, img, pkts[:512], sub, tag="5tuple_call")
    prod = _run(img, pkts, cuda, fixed_stride=64, prod=True)  # the bench's outputs
    _same(prod, got, "5tuple_call prod", keys=("status", "r0", "verdict", "counters"))
