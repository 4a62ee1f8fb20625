"""The reference's own unit tests (src/ins.rs:281-500), restated against the product loader
(ebpf_emu.ins -> libebpfemu.so ebpf_prog_load), and against the oracle and pyref decoders."""
import pytest

from ebpf_emu.ins import (AJ, LS, AOp, Class, DecodeError, HexError, Instruction, JOp, Mode, OP,
                          Register, Source, hexs_to_instructions, hexs_to_u64s, hexs_to_u64s_le,
                          hexs_to_u8s, u64s_to_instructions)

R = Register


def test_hexs_to_u8s():  # ins.rs:291-312
    assert hexs_to_u8s("b7 00  17 ") == [0xB7, 0x00, 0x17]
    with pytest.raises(HexError, match="^invalid hex format$"):
        hexs_to_u8s("b7 00  170 ")
    assert hexs_to_u8s("") == []
    assert hexs_to_u64s("7b  21  02  00  00  00  00  00 ") == [0x7B210200_00000000]
    assert hexs_to_u64s_le("7b  21  02  00  00  00  00  00 ") == [0x00000000_0002217B]
    with pytest.raises(HexError, match="^invalid hex format for u64$"):
        hexs_to_u64s("b7 00 17 ")
    assert hexs_to_u64s("") == []


def test_atomic():  # ins.rs:314-371
    assert hexs_to_instructions("db  1a  f8  ff  a0  00  00  00") == [
        Instruction(0xA0, 0xA0, -8, R.R1, R.R10, LS(Mode.ATOMIC, 24, Class.STX))]
    assert hexs_to_instructions("db  1a  f8  ff  40  00  00  00 ") == [
        Instruction(0x40, 0x40, -8, R.R1, R.R10, LS(Mode.ATOMIC, 0x18, Class.STX))]
    assert hexs_to_instructions("c3  1a  f8  ff  40  00  00  00 ") == [
        Instruction(0x40, 0x40, -8, R.R1, R.R10, LS(Mode.ATOMIC, 0, Class.STX))]


def test_wide():  # ins.rs:373-432
    assert hexs_to_instructions("18  00  00  00  00  00  00  80 00  00  00  00  00  00  00  00") == [
        Instruction(0, 0x80000000, 0, R.R0, R.R0, LS(Mode.IMM, 24, Class.LD))]
    assert hexs_to_instructions("7b  21  02  00  00  00  00  00") == [
        Instruction(0, 0, 2, R.R2, R.R1, LS(Mode.MEM, 24, Class.STX))]
    assert hexs_to_instructions("18  00  00  00  f0  de  bc  9a 00  00  00  00  78  56  34  12") == [
        Instruction(0, 0x123456789ABCDEF0, 0, R.R0, R.R0, LS(Mode.IMM, 24, Class.LD))]


def test_basic_ins():  # ins.rs:433-500 (bpf_conformance/tests/rsh32-imm.data)
    hx = ("b7  00  00  00  00  00  00  00  17  00  00  00  01  00  00  00  74  00  00  00  08  00  00  00"
          "  95  00  00  00  00  00  00  00").strip().replace(" ", "")
    words = [int(hx[i:i + 16], 16) for i in range(0, len(hx), 16)]
    assert u64s_to_instructions(words) == [
        Instruction(0, 0, 0, R.R0, R.R0, AJ(OP.Alu(AOp.MOV), Source.IMM, Class.ALU64)),
        Instruction(1, 1, 0, R.R0, R.R0, AJ(OP.Alu(AOp.SUB), Source.IMM, Class.ALU64)),
        Instruction(8, 8, 0, R.R0, R.R0, AJ(OP.Alu(AOp.RSH), Source.IMM, Class.ALU)),
        Instruction(0, 0, 0, R.R0, R.R0, AJ(OP.Jmp(JOp.EXIT), Source.IMM, Class.JMP)),
    ]


def test_decode_rejects_mirror_panics():
    from cases import REJECTS

    from ebpf_emu.ins import decode_image

    for name, img, code, word, cite in REJECTS:
        with pytest.raises(DecodeError) as ei:
            decode_image(img)
        assert (ei.value.code, ei.value.word) == (code, word), (name, cite)


def test_from_str_radix_plus_sign():
    # u8::from_str_radix accepts a leading '+', as Rust does
    assert hexs_to_u8s("+f0a") == [0x0F, 0x0A]
    with pytest.raises(HexError):
        hexs_to_u8s("zz")


def test_conformance_data_parser():
    """bpf_conformance `.data` parsing (asm and raw forms) agrees with the oracle's answers."""
    import glob
    import os

    import oracle

    from ebpf_emu.conformance import parse_data

    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "conformance")
    files = sorted(glob.glob(os.path.join(d, "*.data")))
    assert len(files) >= 9
    for f in files:
        v = parse_data(open(f).read(), os.path.basename(f))
        st, r0, _ = oracle.Program(v.program).run_packet(v.memory, 1024, 512, 100000)
        if v.expect_error:
            assert st != 0, f
        else:
            assert st == 0 and r0 == v.result, (f, st, hex(r0))
