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


def _images(pkts):
    return [struct.pack("<II", 8, 8 + len(p)) + p for p in pkts]


@pytest.mark.parametrize("layout", [dict(), dict(offsets_layout=True, misalign=3)])
@pytest.mark.parametrize("src", [XDP_PARSE, XDP_SUM])
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
@pytest.mark.parametrize("src", [XDP_PARSE, XDP_SUM])
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
