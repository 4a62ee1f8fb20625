"""Loop mode of the tile interpreter (tile_kernel<..., LOOPS>, csrc/gen_tile.py): programs with back
edges, or with a step budget that can bind, on MI355X. Bit-exact against the C oracle with the
same budget (status of every packet; registers and image of every completing packet; counters
including retired steps), and identical in every output to the general interpreter
(EBPF_BATCH_GENERIC). Covers the two things loop mode adds:
  * the exact step budget: a lane that would run out inside a basic block restarts the tile in
    one-micro-op-per-block mode (emu.rs:452-458 has no limit; ST_STEPS is this build's);
  * the refillable per-lane LDS window: loads past the first 64 bytes, forward, backward and
    strided, in 16-byte aligned (refills) and misaligned (direct packet reads) layouts."""
import random
import zlib

import pytest

from fuzzgen import gen_packet, gen_program
from test_gpu_parity import (_check_against_oracle, _check_prod_against_oracle, _run_full,
                             _run_prod, _same_outputs)

pytestmark = pytest.mark.gpu

# r0 = sum of the packet bytes, forward (workloads.CHECKSUM without the fold)
FORWARD_SUM = """
    mov r0, 0
    mov r3, 0
    jge r3, r2, done
loop:
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    add r0, r5
    add r3, 1
    jlt r3, r2, loop
done:
    exit
"""

# backward scan of 16-bit words (every refill moves the window down)
BACKWARD_WORDS = """
    mov r0, 0
    mov r3, r2
loop:
    jlt r3, 2, done
    sub r3, 2
    mov r4, r1
    add r4, r3
    ldxh r5, [r4+0]
    xor r0, r5
    lsh r0, 1
    ja loop
done:
    exit
"""

# strided 4- and 8-byte reads (r3 = i * 37 mod len), some reading past len (zeros) or past the
# image end (ST_MEM / ST_MEM_UB faults on the lanes whose packets make them do so)
STRIDED = """
    mov r0, 0
    mov r3, 0
    mov r6, 0
loop:
    jge r6, 40, done
    add r6, 1
    add r3, 37
    mov r7, r3
    mod r7, r2
    mov r4, r1
    add r4, r7
    ldxw r5, [r4+0]
    add r0, r5
    ldxdw r5, [r4+3]
    xor r0, r5
    jset r5, 0x100, far
    ja loop
far:
    ldxb r5, [r4+1000]
    add r0, r5
    ja loop
done:
    exit
"""

# byte-only loads (zero windows: the transposed, prefetched refills of jit.cpp refill_prefetch):
# a backward scan (every refill misses the prefetch, which is the window above), a forward scan
# that re-reads byte 0 every 48 bytes (window [0, 64) reloaded, then the forward windows again:
# hits and misses alternate), and strided bytes with reads past len and past the image end
BACKWARD_BYTES = """
    mov r0, 0
    mov r3, r2
loop:
    jle r3, 0, done
    sub r3, 1
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    xor r0, r5
    lsh r0, 1
    ja loop
done:
    exit
"""

REREAD_BYTES = """
    mov r0, 0
    mov r3, 0
    mov r6, 0
loop:
    jge r3, r2, done
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    add r0, r5
    add r3, 1
    add r6, 1
    jlt r6, 48, loop
    mov r6, 0
    ldxb r5, [r1+0]
    xor r0, r5
    ja loop
done:
    exit
"""

STRIDED_BYTES = """
    mov r0, 0
    mov r3, 0
    mov r6, 0
loop:
    jge r6, 40, done
    add r6, 1
    add r3, 37
    mov r7, r3
    mod r7, r2
    mov r4, r1
    add r4, r7
    ldxb r5, [r4+0]
    add r0, r5
    ldxb r5, [r4+70]
    xor r0, r5
    jset r5, 0x4, far
    ja loop
far:
    ldxb r5, [r4+1000]
    add r0, r5
    ja loop
done:
    exit
"""

LOOP_PROGRAMS = [FORWARD_SUM, BACKWARD_WORDS, STRIDED, BACKWARD_BYTES, REREAD_BYTES, STRIDED_BYTES]


def _packets(rng, n):
    lens = [0, 1, 2, 3, 15, 16, 17, 63, 64, 65, 100, 127, 128, 300, 700, 1000]
    return [bytes(rng.getrandbits(8) for _ in range(rng.choice(lens))) for _ in range(n)]


@pytest.mark.parametrize("layout", [dict(), dict(offsets_layout=True, align=16),
                                    dict(offsets_layout=True, misalign=3)])
def test_loop_programs_layouts(cuda, oracle_mod, layout):
    from ebpf_emu.asm import assemble

    rng = random.Random(11)
    pkts = _packets(rng, 150)
    for src in LOOP_PROGRAMS:
        img = assemble(src)
        got = _run_full(img, pkts, cuda, **layout)
        _check_against_oracle(oracle_mod, img, pkts, got, tag=f"{layout} {src[:40]}")
        _same_outputs(got, _run_full(img, pkts, cuda, generic=True, **layout), src)
        prod = _run_prod(img, pkts, cuda, **layout)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, tag=f"prod {layout} {src[:40]}")


@pytest.mark.parametrize("seed", range(3))
def test_fuzz_loop_programs_production_outputs(cuda, oracle_mod, seed):
    """Random tier-0 programs with back edges (the compiled loop kernel) with the production
    outputs only -- no registers, so the liveness-pruned register init runs -- vs the oracle,
    in the stride and offsets + lens layouts."""
    rng = random.Random(6060 + seed)
    n_run = 0
    for it in range(40):
        img = gen_program(rng, allow_loops=True, tier0=True)
        try:
            oracle_mod.Program(img)
        except oracle_mod.OracleDecodeError:
            continue
        pkts = [gen_packet(rng) for _ in range(rng.choice([64, 65, 100, 130]))]
        layout = dict(offsets_layout=True, align=16) if it % 2 else dict()
        prod = _run_prod(img, pkts, cuda, max_steps=2000, **layout)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, max_steps=2000,
                                   tag=f"seed {seed} it {it}")
        n_run += 1
    assert n_run >= 25


@pytest.mark.parametrize("seed", range(2))
def test_fuzz_large_loop_programs(cuda, oracle_mod, seed):
    """Random tier-0 programs of 63-256 micro-ops with back edges: the compiled loop kernel
    (tile_kernel's tables stop at 62) against the oracle (production outputs) and against the
    general interpreter (every output), binding budgets included."""
    from ebpf_emu import Program

    rng = random.Random(7070 + seed)
    n_run = 0
    for it in range(14):
        img = gen_program(rng, n=rng.randrange(70, 250), allow_loops=True, tier0=True)
        try:
            oracle_mod.Program(img)
            p = Program(img)
        except Exception:
            continue
        compiled = p.tier == 0 and p.compile()
        if not compiled:
            p.close()
            continue
        pkts = [gen_packet(rng) for _ in range(rng.choice([64, 65, 100, 130]))]
        layout = dict(offsets_layout=True, align=16) if it % 2 else dict()
        steps = rng.choice([2000, 150])
        # the route: the compiled loop kernel, unless the program is forward-only with a budget
        # that cannot bind (then the compiled forward kernels)
        import torch
        from ebpf_emu import _lib
        frames = torch.zeros(len(pkts) * 256, dtype=torch.uint8, device=cuda)
        k = p.batch_kernel(p.make_batch(frames, n=len(pkts), stride=256, max_steps=steps))
        assert k in (_lib.EBPF_KERNEL_JIT_LOOP, _lib.EBPF_KERNEL_JIT_FIXED,
                     _lib.EBPF_KERNEL_JIT_FIXED_OCC, _lib.EBPF_KERNEL_JIT_VAR,
                     _lib.EBPF_KERNEL_JIT_VARL), _lib.KERNEL_NAMES[k]
        p.close()
        prod = _run_prod(img, pkts, cuda, max_steps=steps, **layout)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, max_steps=steps,
                                   tag=f"seed {seed} it {it}")
        full = _run_full(img, pkts, cuda, max_steps=steps, **layout)
        _same_outputs(full, _run_full(img, pkts, cuda, max_steps=steps, generic=True, **layout),
                      f"seed {seed} it {it} {img.hex()}")
        n_run += 1
    assert n_run >= 6


@pytest.mark.parametrize("budget", [1, 2, 3, 5, 6, 7, 8, 13, 50, 101, 389, 997])
def test_loop_step_budget_exact(cuda, oracle_mod, budget):
    """Budgets that bind at every position of the loop body, for lanes of different lengths in
    one tile: ST_STEPS exactly where the oracle stops (and faults before the budget win)."""
    from ebpf_emu.asm import assemble

    rng = random.Random(budget)
    pkts = _packets(rng, 100)
    for src in LOOP_PROGRAMS:
        img = assemble(src)
        got = _run_full(img, pkts, cuda, max_steps=budget, offsets_layout=True, align=16)
        op = oracle_mod.Program(img)
        retired = 0
        for i, p in enumerate(pkts):
            st, regs, mem, steps = op.run_full(p, 1024, 512, budget)
            assert got["status"][i] == st, (budget, i, src[:40])
            if st == 0:
                assert [int(v) for v in got["regs"][i]] == regs, (budget, i)
            retired += steps
        assert int(got["counters"][7]) == retired, budget
        gen = _run_full(img, pkts, cuda, max_steps=budget, offsets_layout=True, align=16,
                        generic=True)
        _same_outputs(got, gen, f"budget {budget}")
        # the production outputs: the proven copy, whose counted loops (jit.cpp counted_entry)
        # check the budget once per loop entry from the trip count
        prod = _run_prod(img, pkts, cuda, max_steps=budget, offsets_layout=True, align=16)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, max_steps=budget,
                                   tag=f"prod budget {budget} {src[:40]}")


@pytest.mark.parametrize("layout", [dict(offsets_layout=True, align=64),
                                    dict(offsets_layout=True, misalign=5)])
def test_length_binned_batches(cuda, oracle_mod, layout):
    """Batches of >= 16384 packets in the offsets + lens layout run in length-binned order
    (bin_hist / bin_scatter): every output still at its packet's index, identical to the general
    interpreter, and counters equal to the oracle's."""
    import numpy as np

    from ebpf_emu.asm import assemble
    from ebpf_emu import workloads as W

    rng = random.Random(77)
    pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 14, 64, 65, 200, 600, 1500])))
            for _ in range(20000)]
    for src in (W.CHECKSUM, FORWARD_SUM):
        img = assemble(src)
        got = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
        gen = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, generic=True, **layout)
        _same_outputs(got, gen, f"{layout} {src[:30]}")
        (frames, n), kw = _oracle_batch(pkts)
        r0, st, cnt = oracle_mod.Program(img).run_batch(frames, n, mem_size=2048, r10=2048,
                                                        threads=8, **kw)
        assert np.array_equal(got["status"], st)
        assert list(got["counters"]) == [int(c) for c in cnt]


def _oracle_batch(pkts):
    import numpy as np

    buf = b"".join(pkts) + bytes(16)
    offs, pos = [], 0
    for p in pkts:
        offs.append(pos)
        pos += len(p)
    return (np.frombuffer(buf, dtype=np.uint8), len(pkts)), dict(
        offsets=np.array(offs, dtype=np.uint32), lens=np.array([len(p) for p in pkts], dtype=np.uint16))


# Loop programs whose one-byte loads the compiler proves in bounds (jit.cpp prove_loads: the
# index is non-negative and below r2 = the packet length on every path) or must not prove: the
# proven copy drops their bounds checks, so these pin the analysis's edges -- an offset past the
# proof, a `jle` bound (index == len), a negative start (signed compares, Q2), r2 changed in the
# loop, the `jgt r2, r3` form, a 32-bit compare -- on packets as long as the image (mem_size), so
# that every unproven load that overruns faults exactly where the oracle does.
RANGE_PROGRAMS = {
    "proven": FORWARD_SUM,
    "proven_jgt_len": """
    mov r0, 0
    mov r3, 0
    jge r3, r2, done
loop:
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    add r0, r5
    add r3, 1
    jgt r2, r3, loop
done:
    exit
""",
    "off_past_proof": FORWARD_SUM.replace("[r4+0]", "[r4+1]"),
    "jle_bound": FORWARD_SUM.replace("jlt r3, r2, loop", "jle r3, r2, loop"),
    "negative_start": FORWARD_SUM.replace("mov r3, 0", "mov r3, -3"),
    "len_changed": FORWARD_SUM.replace("add r3, 1", "add r3, 1\n    add r2, 1"),
    "jlt32": FORWARD_SUM.replace("jlt r3, r2, loop", "jlt32 r3, r2, loop"),
    "proven_stride2": FORWARD_SUM.replace("add r3, 1", "add r3, 2"),
}


# Counted-loop edges (jit.cpp counted_entry), each a program the compiler takes as a counted loop:
# a trip count of exactly 2^24 (past the 24-bit multiplier that prices the entry's steps); an
# address copy whose register is r0 (an output: the copy must not be dropped); an address copy
# whose source register is rewritten by the block's own load (a later load through the copy must
# not be rebased onto the rewritten register).
COUNTED_EDGE_PROGRAMS = {
    "trip_2p24": """
    mov r3, 0
    mov r6, 0x1000000
    jge r3, r2, loop
    ldxb r5, [r3+0]
loop:
    add r3, 1
    jlt r3, r6, loop
    mov r0, r3
    exit
""",
    "addr_copy_r0": """
    mov r0, 0
    mov r6, 0
    mov r3, 0
    jge r3, r2, done
loop:
    mov r0, r1
    add r0, r3
    ldxb r5, [r0+0]
    add r6, r5
    add r3, 1
    jlt r3, r2, loop
done:
    lsh r6, 32
    add r0, r6
    exit
""",
    "addr_src_loaded": """
    mov r0, 0
    mov r3, 0
    jge r3, r2, done
loop:
    mov r6, r3
    mov r4, r1
    add r4, r6
    ldxb r6, [r4+0]
    ldxb r5, [r4+0]
    add r0, r5
    lsh r0, 1
    add r0, r6
    add r3, 1
    jlt r3, r2, loop
done:
    exit
""",
}


@pytest.mark.parametrize("name", sorted(COUNTED_EDGE_PROGRAMS))
def test_counted_loop_edges(cuda, oracle_mod, name):
    """The counted-loop edges against the oracle, production outputs (the proven copy), at the
    default budget and at budgets around the 2^24-trip loop's exact step count."""
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    img = assemble(COUNTED_EDGE_PROGRAMS[name])
    p = Program(img)
    assert p.compile()
    assert "counted loop" in p.jit_asm(2), name
    p.close()
    rng = random.Random(len(name))
    if name == "trip_2p24":  # (the oracle runs 2^25 steps per packet: a few packets)
        pkts = [bytes(rng.getrandbits(8) for _ in range(n)) for n in (0, 14, 64)]
        steps = 6 + 2 * (1 << 24)  # the whole run of a non-empty packet (5 + ... when empty)
        for budget in (1 << 22, steps - 1, steps):
            prod = _run_prod(img, pkts, cuda, max_steps=budget)
            _check_prod_against_oracle(oracle_mod, img, pkts, prod, max_steps=budget,
                                       tag=f"{name} budget {budget}")
        assert (prod["status"] == 0).all() and (prod["r0"] == 1 << 24).all()
        return
    pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 9, 63, 64, 65, 300, 700])))
            for _ in range(200)]
    for layout in (dict(), dict(offsets_layout=True, align=16)):
        prod = _run_prod(img, pkts, cuda, **layout)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, tag=f"{name} {layout}")


def gen_scan_program(rng):
    """A random byte scan: r3 from a start value, step, guard and back-edge compare drawn from
    forms the range analysis proves or must refuse (offsets past the proof, <= bounds, negative
    starts, constant bounds, r2 rewritten), loads [r1 + r3 + off]."""
    ok = rng.random() < 0.5  # half from the provable forms only
    start = rng.choice([0, 1, 3] + ([] if ok else [-1, -5]))
    step = rng.choice([1, 1, 2, 3])
    off = rng.choice([0] if ok else [0, 1, 2, -1])
    guard = rng.choice(["jge r3, r2, done", "jle r2, r3, done"] +
                       ([] if ok else ["jge r3, 40, done", ""]))
    back = rng.choice(["jlt r3, r2, loop", "jgt r2, r3, loop"] +
                      ([] if ok else ["jle r3, r2, loop", "jge r2, r3, loop", "jne r3, r2, loop",
                                      "jlt r3, 40, loop", "jlt32 r3, r2, loop"]))
    extra = rng.choice(["", "and r3, 0x3f"] + ([] if ok else ["add r2, 1", "mov r2, 200"]))
    return f"""
    mov r0, 0
    mov r3, {start}
    {guard}
loop:
    mov r4, r1
    add r4, r3
    ldxb r5, [r4{off:+d}]
    add r0, r5
    {extra}
    add r3, {step}
    {back}
done:
    exit
"""


@pytest.mark.parametrize("seed", range(2))
def test_fuzz_range_proofs(cuda, oracle_mod, seed):
    """Random byte scans (gen_scan_program), proven or not, on packets as long as the image:
    the production outputs (the proven copy) and the full outputs (the checked copy) against the
    oracle, status of every packet included."""
    from ebpf_emu.asm import assemble

    rng = random.Random(8080 + seed)
    for it in range(24):
        img = assemble(gen_scan_program(rng))
        mem = rng.choice([64, 96])
        pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 5, mem - 2, mem, mem])))
                for _ in range(130)]
        prod = _run_prod(img, pkts, cuda, mem_size=mem, max_steps=3000)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, mem_size=mem, max_steps=3000,
                                   tag=f"seed {seed} it {it}")


@pytest.mark.parametrize("name", sorted(RANGE_PROGRAMS))
def test_loop_range_proofs(cuda, oracle_mod, name):
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    img = assemble(RANGE_PROGRAMS[name])
    p = Program(img)
    assert p.compile()
    proven = "one-byte loads proven in bounds" in p.jit_asm(2)
    p.close()
    assert proven == name.startswith("proven"), name
    rng = random.Random(zlib.crc32(name.encode()))
    for mem in (64, 128):
        pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 17, mem - 1, mem, mem])))
                for _ in range(200)]
        for layout in (dict(), dict(offsets_layout=True, align=16)):
            prod = _run_prod(img, pkts, cuda, mem_size=mem, **layout)
            _check_prod_against_oracle(oracle_mod, img, pkts, prod, mem_size=mem,
                                       tag=f"{name} mem {mem} {layout}")
            got = _run_full(img, pkts, cuda, mem_size=mem, **layout)
            _check_against_oracle(oracle_mod, img, pkts, got, mem_size=mem,
                                  tag=f"full {name} mem {mem} {layout}")


def gen_group_program(rng):
    """A counted byte scan of the grouped form (jit.cpp counted_group: one `ldxb` from r3, r3
    stepped by one, back edge `jlt r3, r2`): starts that differ per lane (misaligned passes), a
    body that reads r3 itself (no folded increment) or not, and a tail that folds the final r3
    and r5 into r0 so the production outputs see them."""
    start = rng.choice(["mov r3, 0", "mov r3, 3", "mov r3, 8",
                        "ldxb r3, [r1+0]\n    and r3, 7", "ldxb r3, [r1+1]\n    and r3, 15"])
    base = rng.choice(["mov r4, r1\n    add r4, r3\n    ldxb r5, [r4+0]", "ldxb r5, [r3+0]"])
    mix = rng.choice(["add r0, r5", "xor r0, r5\n    lsh r0, 1", "add r0, r5\n    xor r0, r3",
                      "mov r6, r5\n    lsh r6, 3\n    sub r0, r6", "add32 r0, r5", "add r0, r5"])
    pre = rng.choice(["", "mov r5, -1", "mov r5, 0x1234"])
    # the block's other micro-ops after the load, or before it (then they see the previous
    # iteration's byte: not the byte-sum idiom)
    body = f"{base}\n    {mix}" if rng.random() < 0.7 else f"{mix}\n    {base}"
    return f"""
    mov r0, 0
    {pre}
    {start}
    jge r3, r2, done
loop:
    {body}
    add r3, 1
    jlt r3, r2, loop
done:
    mov r6, r5
    lsh r6, 8
    xor r0, r6
    xor r0, r3
    exit
"""


@pytest.mark.parametrize("seed", range(2))
def test_counted_loop_passes(cuda, oracle_mod, seed):
    """Counted loops run 8 iterations per pass from one qword of the window (counted_group):
    packets of every length up to 700 bytes (passes, refills, remainders of 0..7, packets shorter
    than one pass), per-lane starts that differ mod 8, 16-byte aligned and unaligned packet bases
    (no refills: the far path); production outputs and step counters against the oracle."""
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    rng = random.Random(4242 + seed)
    for it in range(10):
        src = gen_group_program(rng)
        img = assemble(src)
        p = Program(img)
        assert p.compile()
        assert "8 per pass" in p.jit_asm(2), src
        p.close()
        pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 3, 8, 9, 63, 64, 65, 71,
                                                                    rng.randrange(700)])))
                for _ in range(300)]
        for layout in (dict(), dict(offsets_layout=True, align=16),
                       dict(offsets_layout=True, align=1, misalign=3)):
            prod = _run_prod(img, pkts, cuda, mem_size=1024, max_steps=100000, **layout)
            _check_prod_against_oracle(oracle_mod, img, pkts, prod, mem_size=1024,
                                       max_steps=100000, tag=f"seed {seed} it {it} {layout}")


# Byte scans for the refill prefetch (jit.cpp refill_prefetch): sequential windows (lockstep
# lanes hit their prefetched window), strides that skip windows (every refill a miss: the window
# loaded directly), a backward scan, and lengths that differ per lane.
DEEP_SCANS = [FORWARD_SUM] + [FORWARD_SUM.replace("add r3, 1", f"add r3, {s}") for s in (5, 64, 100, 130)] + [
    """
    mov r0, 0
    mov r3, r2
    jeq r3, 0, done
loop:
    sub r3, 1
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    add r0, r5
    lsh r0, 1
    jgt r3, 0, loop
done:
    exit
"""]


def test_prefetch_scans(cuda, oracle_mod):
    """The refill prefetch over the checksum and byte scans with window-skipping strides, a
    backward scan and per-lane lengths, binned and unbinned batches, two alignments of the
    offsets layout -- compiled == general interpreter == oracle."""
    import numpy as np

    from ebpf_emu import Program
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    depth = 1
    rng = random.Random(zlib.crc32(b"prefetch"))
    for i, src in enumerate([W.CHECKSUM] + DEEP_SCANS):
        img = assemble(src)
        p = Program(img)
        assert p.compile()
        assert "global_load_dwordx4 v[56:59]" in p.jit_asm(2), src
        p.close()
        n = 17000 if i < 2 else 700  # (>= 16384: length-binned order)
        lens = [rng.choice([0, 14, 64, 65, 200, 600, 1500, 1500, 1500, rng.randrange(1501)])
                for _ in range(n)]
        pkts = [bytes(rng.getrandbits(8) for _ in range(ln)) for ln in lens]
        for layout in (dict(offsets_layout=True, align=16), dict(offsets_layout=True, align=64)):
            got = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
            gen = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, generic=True, **layout)
            _same_outputs(got, gen, f"depth {depth} {layout} {src[:40]}")
            (frames, nn), kw = _oracle_batch(pkts)
            r0, st, cnt = oracle_mod.Program(img).run_batch(frames, nn, mem_size=2048, r10=2048,
                                                            threads=8, **kw)
            assert np.array_equal(got["status"], st)
            assert np.array_equal(got["r0"], np.asarray(r0, dtype=np.uint64))
            assert list(got["counters"]) == [int(c) for c in cnt]
            prod = _run_prod(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
            assert np.array_equal(prod["r0"], got["r0"]) and np.array_equal(prod["status"], st)
            assert list(prod["counters"]) == list(got["counters"])


W_CHECKSUM_BODY = """
    mov r0, 0
    {pre}
    {start}
    jge r3, r2, done
loop:
    {load}
    add r0, r5
    add r3, 1
    jlt r3, r2, loop
done:
    mov r6, r5
    lsh r6, 8
    xor r0, r6
    xor r0, r3
    exit
"""


# Byte-sum loops for coop_sum (jit.cpp: the sum of a whole range, transposed, from HBM): starts
# that are not 16-aligned, a load offset (d != 0), rD with its upper bytes set (n * (rD & ~0xff)),
# a 32-bit sum register... and lengths around kCoopMin (128) and up to 1500.
COOP_PROGRAMS = {
    "sum": W_CHECKSUM_BODY.format(pre="", start="mov r3, 0", load="ldxb r5, [r3+0]"),
    "start5_upper": W_CHECKSUM_BODY.format(pre="lddw r5, 0x123456789abcde00", start="mov r3, 5",
                                           load="ldxb r5, [r3+0]"),
    "addr_copy": W_CHECKSUM_BODY.format(pre="mov r5, -1", start="ldxb r3, [r1+0]\n    and r3, 31",
                                        load="mov r4, r1\n    add r4, r3\n    ldxb r5, [r4+0]"),
    "offset": """
    mov r0, 7
    mov r3, 0
    mov r6, r2
    sub r6, 3
    jsge r3, r6, done
loop:
    ldxb r5, [r3+2]
    add r0, r5
    add r3, 1
    jlt r3, r6, loop
done:
    xor r0, r5
    lsh r5, 9
    xor r0, r5
    xor r0, r3
    exit
""",
}


@pytest.mark.parametrize("name", sorted(COOP_PROGRAMS))
def test_coop_byte_sum(cuda, oracle_mod, name):
    """Counted byte-sum loops whose long ranges are summed cooperatively (coop_sum_compact on the
    deep kernel): production and full outputs against the oracle on packets of 0-1500 bytes
    (lengths around the 128-byte threshold included), aligned and misaligned packet bases, binned
    and unbinned batches."""
    import numpy as np

    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    img = assemble(COOP_PROGRAMS[name])
    p = Program(img)
    assert p.compile()
    a = p.jit_asm(2)
    coop = "coop_sum" in a
    p.close()
    if name != "offset":
        assert coop, name
        assert "coop_sum_compact" in a, name
    rng = random.Random(zlib.crc32(name.encode()))
    for n in (700, 17000):
        lens = [rng.choice([0, 1, 127, 128, 129, 130, 143, 144, 200, 1500, 1500, rng.randrange(1501)])
                for _ in range(n)]
        pkts = [bytes(rng.getrandbits(8) for _ in range(ln)) for ln in lens]
        for layout in (dict(offsets_layout=True, align=16), dict(offsets_layout=True, misalign=5)):
            prod = _run_prod(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
            (frames, nn), kw = _oracle_batch(pkts)
            r0, st, cnt = oracle_mod.Program(img).run_batch(frames, nn, mem_size=2048, r10=2048,
                                                            threads=8, **kw)
            assert np.array_equal(prod["status"], st), (name, n, layout)
            assert np.array_equal(prod["r0"], np.asarray(r0, dtype=np.uint64)), (name, n, layout)
            assert list(prod["counters"]) == [int(c) for c in cnt], (name, n, layout)
            if n == 700:
                full = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
                gen = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, generic=True, **layout)
                _same_outputs(full, gen, f"{name} {layout}")


@pytest.mark.parametrize("name", ["sum", "start5_upper", "addr_copy"])
def test_coop_compact_tile_densities(cuda, oracle_mod, name):
    """coop_sum_compact picks 16, 8 or 4 lanes per packet from the number C of cooperating lanes
    in a tile (C <= 16, <= 32, > 32): batch-order tiles with exactly C long packets (1..64, at
    random positions, lengths 128-1500) among short ones, C across every threshold; production
    outputs against the oracle, aligned and misaligned bases."""
    import numpy as np

    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    img = assemble(COOP_PROGRAMS[name])
    p = Program(img)
    assert p.compile()
    assert "coop_sum_compact" in p.jit_asm(2)
    p.close()
    rng = random.Random(zlib.crc32(b"density" + name.encode()))
    lens = []
    for c in (1, 2, 15, 16, 17, 31, 32, 33, 48, 63, 64, 0, 5, 40):
        tile = [rng.randrange(129, 1501) if i < c else rng.choice([0, 1, 64, 127, 128])
                for i in range(64)]
        rng.shuffle(tile)
        lens += tile
    pkts = [bytes(rng.getrandbits(8) for _ in range(ln)) for ln in lens]
    for layout in (dict(offsets_layout=True, align=16), dict(offsets_layout=True, misalign=3)):
        prod = _run_prod(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
        (frames, nn), kw = _oracle_batch(pkts)
        r0, st, cnt = oracle_mod.Program(img).run_batch(frames, nn, mem_size=2048, r10=2048,
                                                        threads=8, **kw)
        assert np.array_equal(prod["status"], st), (name, layout)
        assert np.array_equal(prod["r0"], np.asarray(r0, dtype=np.uint64)), (name, layout)
        assert list(prod["counters"]) == [int(c) for c in cnt], (name, layout)
        full = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
        assert np.array_equal(full["r0"], prod["r0"]) and np.array_equal(full["status"], st)


@pytest.mark.parametrize("name", ["sum", "start5_upper"])
def test_coop_budget_edges(cuda, oracle_mod, name):
    """Step budgets around what the longest cooperating packets need (coop_sum_compact runs under
    a budget the counted entry proved sufficient; one step less must end in ST_STEPS exactly
    where the oracle stops): budgets = the largest packet's steps, one less, and the median --
    production outputs, verdicts and counters against the oracle."""
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    img = assemble(COOP_PROGRAMS[name])
    p = Program(img)
    assert p.compile() and "coop_sum_compact" in p.jit_asm(2)
    p.close()
    rng = random.Random(zlib.crc32(b"budget" + name.encode()))
    lens = [rng.choice([64, 127, 128, 600, 1499, 1500, rng.randrange(129, 1501)]) for _ in range(640)]
    pkts = [bytes(rng.getrandbits(8) for _ in range(ln)) for ln in lens]
    op = oracle_mod.Program(img)
    steps = sorted(op.run_packet(q, 2048, 2048, 1 << 22)[2] for q in pkts)
    for budget in (steps[-1], steps[-1] - 1, steps[len(steps) // 2]):
        prod = _run_prod(img, pkts, cuda, mem_size=2048, r10=2048, max_steps=budget,
                         offsets_layout=True, align=16)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, mem_size=2048, r10=2048,
                                   max_steps=budget, tag=f"{name} budget {budget}")


def gen_bytesum_program(rng):
    """A random counted byte-sum loop around the shape coop_sum takes (and near misses): random
    accumulator / byte / index / bound registers, start (constant or a packet byte), bound (len,
    len - c), load offset d (at most c: in bounds, or more: some lanes fault), base direct or an
    address copy, accumulator and byte register preloaded with random 64-bit values, a 32-bit add
    or an add before the load now and then (not the idiom), and an epilogue that mixes every
    register the loop leaves into r0."""
    S = rng.choice(["r0", "r6", "r7"])
    D = rng.choice(["r5", "r8"])
    I = rng.choice(["r3", "r4"])
    A = "r4" if I == "r3" else "r3"
    # bound: len (unsigned), len >> 1 (unsigned), or len - c (signed compares; not a counted loop)
    bk = rng.choices(["len", "half", "sub"], weights=[5, 2, 2])[0]
    N = "r2" if bk == "len" else "r9"
    c = rng.choice([0, 1, 2, 3, 7])
    d = {"len": 0, "half": rng.choice([0, 0, 3]), "sub": rng.choice([0, 0, 1, 2, c, c + 1])}[bk]
    lines = [f"lddw {S}, {rng.getrandbits(64):#x}" if rng.random() < 0.5 else f"mov {S}, {rng.randrange(100)}",
             f"lddw {D}, {rng.getrandbits(64):#x}"]
    if rng.random() < 0.7:
        lines.append(f"mov {I}, {rng.choice([0, 0, 1, 5, 16, 33])}")
    else:
        lines += [f"ldxb {I}, [r1+{rng.randrange(8)}]", f"and {I}, {rng.choice([15, 31, 63])}"]
    if bk == "sub":
        lines += ["mov r9, r2", f"sub r9, {c}"]
    elif bk == "half":
        lines += ["mov r9, r2", "rsh r9, 1"]
    signed = bk == "sub"
    lines.append(f"{'jsge' if signed else 'jge'} {I}, {N}, done")
    lines.append("loop:")
    body = []
    if rng.random() < 0.5:
        body += [f"mov {A}, r1", f"add {A}, {I}", f"ldxb {D}, [{A}+{d}]"]
    else:
        body.append(f"ldxb {D}, [{I}+{d}]")
    r = rng.random()
    if r < 0.1:
        body.append(f"add32 {S}, {D}")          # not the 64-bit idiom
    elif r < 0.15:
        body.insert(0, f"add {S}, {D}")         # the add before the load: the previous byte
    else:
        body.append(f"add {S}, {D}")
    body.append(f"add {I}, 1")
    lines += body
    lines.append(f"{'jslt' if signed else 'jlt'} {I}, {N}, loop")
    lines.append("done:")
    if S != "r0":
        lines.append(f"mov r0, {S}")
    k = rng.randrange(1, 40)
    lines += [f"xor r0, {D}", f"lsh {D}, {k}", f"xor r0, {D}", f"xor r0, {I}", f"mov r9, {I}",
              f"rsh r9, 3", "add r0, r9"]
    if rng.random() < 0.5:
        lines += ["mov r6, r0", "rsh r6, 8", "xor r0, r6", "and r0, 7"]
    lines.append("exit")
    return "\n".join("    " + ln if not ln.endswith(":") else ln for ln in lines) + "\n"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_bytesum_loops(cuda, oracle_mod, seed):
    """Random counted byte-sum loops (gen_bytesum_program) over packets of 0-1500 bytes, in batch
    order (the deep kernel's compacted cooperative sums) and aligned / misaligned bases: production
    outputs against the oracle, full outputs against the general interpreter for some; at least a
    quarter of the programs take coop_sum."""
    from ebpf_emu import Program
    from ebpf_emu.asm import assemble

    rng = random.Random(1000 + seed)
    n_coop = 0
    n_prog = 30
    for it in range(n_prog):
        src = gen_bytesum_program(rng)
        img = assemble(src)
        p = Program(img)
        assert p.compile(), src
        n_coop += "coop_sum" in p.jit_asm(2)
        p.close()
        lens = [rng.choice([0, 1, 5, 64, 127, 128, 129, 200, 700, 1500, rng.randrange(1501)])
                for _ in range(rng.choice([300, 700]))]
        pkts = [bytes(rng.getrandbits(8) for _ in range(ln)) for ln in lens]
        layout = rng.choice([dict(offsets_layout=True, align=16), dict(offsets_layout=True, align=64),
                             dict(offsets_layout=True, misalign=3)])
        prod = _run_prod(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
        _check_prod_against_oracle(oracle_mod, img, pkts, prod, mem_size=2048, r10=2048,
                                   tag=f"seed {seed} it {it}\n{src}")
        if it % 4 == 0:
            full = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, **layout)
            gen = _run_full(img, pkts, cuda, mem_size=2048, r10=2048, generic=True, **layout)
            _same_outputs(full, gen, f"seed {seed} it {it}\n{src}")
    assert n_coop * 4 >= n_prog, n_coop
