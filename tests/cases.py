"""Directed known-answer cases: the reference's embedded KATs, the behaviours its comments quote
from bpf_conformance, and one case (or more) per semantic quirk Q1-Q26 of SURVEY.md §8a.

Expected values were derived by reading the reference source (cited per case); they are NOT
outputs of the Rust reference, which cannot run here. Each case is checked against the C
oracle, the independent Python restatement and (on the GPU box) the HIP kernel.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ebpf_emu.asm import assemble, encode, lddw

OK, MEM, MEM_UB, INSN, ARITH, STEPS, CALLDEPTH, BADPKT = range(8)
M64 = (1 << 64) - 1


@dataclass
class Case:
    name: str
    prog: bytes
    pkt: bytes = b""
    status: int = OK
    r0: int | None = None          # expected r0 (u64) when status == OK
    cite: str = ""
    mem_size: int = 1024
    r10: int = 512
    max_steps: int = 0             # 0 = unlimited (oracle); GPU uses a default budget
    extra: dict = field(default_factory=dict)


def h(s: str) -> bytes:
    return bytes.fromhex(s.replace(" ", ""))


A = assemble

CASES = [
    # ---- reference-embedded KATs ----
    Case("kat_rsh32_imm", h("b7 00 00 00 00 00 00 00 17 00 00 00 01 00 00 00 74 00 00 00 08 00 00 00"
                            " 95 00 00 00 00 00 00 00"), r0=0xFFFFFF, cite="ins.rs:435 (rsh32-imm.data)"),
    Case("kat_stxb", h("b4 02 00 00 11 00 00 00 73 21 02 00 00 00 00 00 71 10 02 00 00 00 00 00"
                       " 95 00 00 00 00 00 00 00"), pkt=h("aa bb ff cc dd"), r0=0x11, cite="notes.md:27"),
    Case("kat_lock_cmpxchg32", h(
        "18 00 00 00 f0 de bc 9a 00 00 00 00 78 56 34 12 7b 0a f8 ff 00 00 00 00 b4 01 00 00 10 32 54 76"
        " b4 00 00 00 78 56 34 12 c3 1a f8 ff f1 00 00 00 b4 01 00 00 f0 de bc 9a 5d 10 10 00 00 00 00 00"
        " 79 a0 f8 ff 00 00 00 00 18 01 00 00 f0 de bc 9a 00 00 00 00 78 56 34 12 5d 10 0c 00 00 00 00 00"
        " 18 00 00 00 f0 de bc 9a 00 00 00 00 78 56 34 12 7b 0a f8 ff 00 00 00 00 b4 01 00 00 44 33 22 11"
        " c3 1a f8 ff f1 00 00 00 b4 01 00 00 f0 de bc 9a 5d 10 05 00 00 00 00 00 79 a0 f8 ff 00 00 00 00"
        " 18 01 00 00 44 33 22 11 00 00 00 00 78 56 34 12 5d 10 01 00 00 00 00 00 b7 00 00 00 00 00 00 00"
        " 95 00 00 00 00 00 00 00"), r0=0, cite="Makefile:16 (lock_cmpxchg32.data)"),
    # ---- behaviours the reference's comments quote from bpf_conformance ----
    Case("arsh32_imm_high", A("mov32 r0, 0x80000000\narsh32 r0, 48\nexit"), r0=0xFFFF8000,
         cite="emu.rs:150-155 (arsh32-imm-high.data)"),
    Case("lsh32_reg_neg", A("mov r0, 0x11\nmov r3, -4\nlsh32 r0, r3\nexit"), r0=0x10000000,
         cite="emu.rs:108-111 (lsh32-reg-neg.data)"),
    Case("div32_by_zero_reg", A("mov32 r0, 7\nmov32 r3, 0\ndiv32 r0, r3\nexit"), r0=0,
         cite="emu.rs:96-98 (div32-by-zero-reg.data)"),
    Case("mod64_by_zero_reg", A("mov r0, 7\nmov r3, 0\nmod r0, r3\nexit"), r0=7,
         cite="emu.rs:130-133 (mod64-by-zero-reg.data)"),
    Case("mem_len", A("mov r0, r2\nexit"), pkt=bytes(5), r0=5, cite="main.rs:26-28 (mem-len.data)"),
    # ---- Q1 LDX sub-width preserves the upper bytes (emu.rs:341-349,443) ----
    Case("q1_ldxb", A("lddw r0, 0x1122334455667788\nldxb r0, [r1+0]\nexit"), pkt=h("aa"),
         r0=0x11223344556677AA, cite="emu.rs:341-349"),
    Case("q1_ldxh", A("lddw r0, 0x1122334455667788\nldxh r0, [r1+0]\nexit"), pkt=h("aa bb"),
         r0=0x112233445566BBAA, cite="emu.rs:341-349"),
    Case("q1_ldxw_unaligned", A("lddw r0, 0x1122334455667788\nldxw r0, [r1+1]\nexit"),
         pkt=h("00 aa bb cc dd"), r0=0x11223344DDCCBBAA, cite="emu.rs:341-349"),
    Case("q1_ldxdw", A("lddw r0, 0x1122334455667788\nldxdw r0, [r1+3]\nexit"),
         pkt=h("00 00 00 01 02 03 04 05 06 07 08"), r0=0x0807060504030201, cite="emu.rs:341-349"),
    # ---- Q2 unsigned-named jumps compare signed (emu.rs:234-299) ----
    Case("q2_jgt_signed", A("mov r3, -1\nmov r0, 0\njgt r3, 1, +1\nmov r0, 1\nexit"), r0=1,
         cite="emu.rs:234-238"),
    Case("q2_jlt_signed", A("mov r3, -1\nmov r0, 0\njlt r3, 1, +1\nmov r0, 1\nexit"), r0=0,
         cite="emu.rs:280-284"),
    Case("q2_jge_reg", A("mov r3, -2\nmov r4, 3\nmov r0, 0\njge r3, r4, +1\nmov r0, 1\nexit"), r0=1,
         cite="emu.rs:239-244"),
    Case("q2_jle_reg", A("mov r3, -2\nmov r4, 3\nmov r0, 0\njle r3, r4, +1\nmov r0, 1\nexit"), r0=0,
         cite="emu.rs:285-289"),
    # ---- Q3 JMP32 sign-extends the low words (emu.rs:221-224) ----
    Case("q3_jgt32", A("lddw r3, 0x00000001FFFFFFFF\nmov r0, 0\njgt32 r3, 0, +1\nmov r0, 1\nexit"),
         r0=1, cite="emu.rs:221-224"),
    Case("q3_jeq32_high_bits", A("lddw r3, 0x0000000100000005\nmov r0, 0\njeq32 r3, 5, +1\nmov r0, 1\nexit"),
         r0=0, cite="emu.rs:221-224"),
    Case("q3_jset32", A("lddw r3, 0xFFFFFFFF00000000\nmov r0, 0\njset32 r3, -1, +1\nmov r0, 1\nexit"),
         r0=1, cite="emu.rs:245-249"),
    # ---- Q4 ARSH = rotate x sign (emu.rs:142-164) ----
    Case("q4_arsh64_neg", A("lddw r0, 0x8000000000000001\narsh r0, 1\nexit"), r0=0x4000000000000000,
         cite="emu.rs:161-162"),
    Case("q4_arsh64_pos_rotates", A("mov r0, 1\narsh r0, 1\nexit"), r0=0x8000000000000000,
         cite="emu.rs:161-162"),
    Case("q4_arsh32_reg", A("mov32 r0, 0xF0000001\nmov r3, 4\narsh32 r0, r3\nexit"), r0=0xE1000000,
         cite="emu.rs:156-159"),
    # ---- Q5 div0 -> 0, mod0 -> unchanged; unsigned (emu.rs:90-135) ----
    Case("q5_div_imm0", A("mov r0, 9\ndiv r0, 0\nexit"), r0=0, cite="emu.rs:96-98"),
    Case("q5_mod32_reg0", A("mov r0, -9\nmov r3, 0\nmod32 r0, r3\nexit"), r0=0xFFFFFFF7,
         cite="emu.rs:76-79,130-133,214-216"),
    Case("q5_div_unsigned", A("mov r0, -4\ndiv r0, 2\nexit"), r0=0x7FFFFFFFFFFFFFFE, cite="emu.rs:95"),
    Case("q5_mod_unsigned", A("mov r0, -1\nmod r0, 10\nexit"), r0=(M64 % 10), cite="emu.rs:129"),
    # ---- Q6/Q25 ALU32 truncation ----
    Case("q6_add32", A("lddw r0, 0x0000000100000001\nadd32 r0, 1\nexit"), r0=2, cite="emu.rs:76-79"),
    Case("q6_mov32_neg", A("mov32 r0, -1\nexit"), r0=0xFFFFFFFF, cite="emu.rs:214-216"),
    Case("q25_mul32", A("mov32 r0, -1\nmov32 r3, -1\nmul32 r0, r3\nexit"), r0=1, cite="emu.rs:87-89"),
    Case("q6_neg32", A("mov r0, 1\nneg32 r0\nexit"), r0=0xFFFFFFFF, cite="emu.rs:125"),
    Case("q6_neg64", A("mov r0, 1\nneg r0\nexit"), r0=M64, cite="emu.rs:125"),
    # ---- Q7 END by source bit, either ALU class (emu.rs:165-209) ----
    Case("q7_le16", A("lddw r0, 0x1122334455667788\nle16 r0\nexit"), r0=0x7788, cite="emu.rs:171-176"),
    Case("q7_be16", A("lddw r0, 0x1122334455667788\nbe16 r0\nexit"), r0=0x8877, cite="emu.rs:177-180"),
    Case("q7_le32", A("lddw r0, 0x1122334455667788\nle32 r0\nexit"), r0=0x55667788, cite="emu.rs:185-188"),
    Case("q7_be32", A("lddw r0, 0x1122334455667788\nbe32 r0\nexit"), r0=0x88776655, cite="emu.rs:189-192"),
    Case("q7_le64", A("lddw r0, 0x1122334455667788\nle64 r0\nexit"), r0=0x1122334455667788,
         cite="emu.rs:197-199"),
    Case("q7_be64", A("lddw r0, 0x1122334455667788\nbe64 r0\nexit"), r0=0x8877665544332211,
         cite="emu.rs:200-202"),
    Case("q7_be16_alu64_class", lddw(0, 0x1122334455667788) + encode(0xDF, 0, 0, 0, 16) + encode(0x95),
         r0=0x8877, cite="emu.rs:74,165 (END for class ALU64)"),
    Case("q7_end_bad_imm", A("mov r0, 1") + encode(0xD4, 0, 0, 0, 8) + encode(0x95), status=INSN,
         cite="emu.rs:205-207"),
    # ---- Q8 ST stores the zero-extended imm (emu.rs:319,356) ----
    Case("q8_stdw_imm", A("stdw [r10-8], -1\nldxdw r0, [r10-8]\nexit"), r0=0xFFFFFFFF, cite="ins.rs:125"),
    # ---- Q9 lddw is one decoded entry for jump offsets (ins.rs:107-116) ----
    Case("q9_ja_over_lddw", A("ja +1\nlddw r0, 5\nmov r0, 7\nexit"), r0=7, cite="ins.rs:107-116, emu.rs:227"),
    Case("q9_ja_to_exit", encode(0x05, 0, 0, 2) + lddw(0, 5) + encode(0xB7, 0, 0, 0, 7) + encode(0x95),
         r0=0, cite="ins.rs:107-116"),
    # ---- Q10 every LS mode-0 opcode is wide; second word's low bits are added ----
    Case("q10_ldx_imm_wide", encode(0x19, 0, 0, 0, 5) + (0x0000000300000007).to_bytes(8, "little")
         + encode(0x95), r0=0x30000000C, cite="ins.rs:107-114"),
    Case("q10_st_imm_wide_faults", encode(0x1A, 0, 0, 0, 5) + bytes(8) + encode(0x95), status=INSN,
         cite="ins.rs:107-114, emu.rs:438"),
    # ---- Q11 falling off the end / jumping out of range stops normally ----
    Case("q11_fall_off", A("mov r0, 3"), r0=3, cite="emu.rs:49,448-450"),
    Case("q11_jump_far", A("mov r0, 4\nja +100\nmov r0, 5\nexit"), r0=4, cite="emu.rs:49,227"),
    Case("q11_jump_wrap", A("mov r0, 6\nja -5\nexit"), r0=6, cite="emu.rs:227 wrapping_add_signed"),
    Case("q11_empty", b"", r0=0, cite="emu.rs:49"),
    # ---- Q12 CALL pushes target+1 and jumps by off; EXIT pops (emu.rs:265-279) ----
    Case("q12_call", A("mov r0, 1\ncall +2\nadd r0, 10\nexit\nadd r0, 100\nexit"), r0=101,
         cite="emu.rs:265-279"),
    Case("q12_call_ret_into_body", A("mov r0, 1\ncall +1\nexit\nadd r0, 2\nadd r0, 4\nexit"), r0=11,
         cite="emu.rs:267-268,275"),
    Case("q12_callx_faults", encode(0x8D, 0, 1, 0, 0) + encode(0x95), status=INSN, cite="emu.rs:269-271"),
    Case("q12_call_depth", A("call -1"), status=CALLDEPTH, cite="emu.rs:268 (unbounded Vec)"),
    # ---- Q13 atomic32: carry leaks into the high word; 8-byte footprint (emu.rs:373-437) ----
    Case("q13_add32_carry", A("lddw r3, 0x00000001FFFFFFFF\nstxdw [r10-8], r3\nmov r4, 1\n"
                              "lock add32 [r10-8], r4\nldxdw r0, [r10-8]\nexit"), r0=0x200000000,
         cite="emu.rs:382-389,427-428"),
    Case("q13_atomic32_footprint", A("mov r4, 1\nlock add32 [r1+1020], r4\nexit"), status=MEM,
         cite="emu.rs:375 read::<i64>"),
    Case("q13_fetch_or32", A("lddw r3, 0x1111111100000001\nstxdw [r10-8], r3\nmov r4, 6\n"
                             "lock fetch or32 [r10-8], r4\nldxdw r0, [r10-8]\nadd r0, r4\nexit"),
         r0=0x1111111100000007 + 1, cite="emu.rs:395-397,433-436"),
    Case("q13_xchg", A("mov r3, 21\nstxdw [r10-8], r3\nmov r4, 5\nlock xchg [r10-8], r4\n"
                       "ldxdw r0, [r10-8]\nlsh r0, 8\nor r0, r4\nexit"), r0=(5 << 8) | 21,
         cite="emu.rs:404-408"),
    Case("q13_xor_nofetch", A("mov r3, 12\nstxdw [r10-8], r3\nmov r4, 10\nlock xor [r10-8], r4\n"
                              "ldxdw r0, [r10-8]\nexit"), r0=6, cite="emu.rs:401-403"),
    Case("q13_and", A("mov r3, 12\nstxdw [r10-8], r3\nmov r4, 10\nlock and [r10-8], r4\n"
                      "ldxdw r0, [r10-8]\nexit"), r0=8, cite="emu.rs:398-400"),
    Case("q13_cmpxchg_nofetch_r0_zero",
         A("mov r3, 4\nstxdw [r10-8], r3\nmov r0, 4\nmov r4, 9\n") +
         encode(0xDB, 10, 4, -8, 0xF0) + A("lsh r0, 8\nldxdw r5, [r10-8]\nor r0, r5\nexit"),
         r0=9, cite="emu.rs:377,409-419 (bak = 0 without fetch)"),
    Case("q13_unknown_atomic", A("mov r4, 1") + encode(0xDB, 10, 4, -8, 0x10) + encode(0x95),
         status=INSN, cite="emu.rs:420-425"),
    Case("q13_unknown_atomic_oob_first", A("mov r4, 1") + encode(0xDB, 1, 4, 2000, 0x10) + encode(0x95),
         status=MEM, cite="emu.rs:375 before :421"),
    # ---- Q14 the dst snapshot write-back clobbers fetch / r0 results (emu.rs:443) ----
    Case("q14_fetch_src_eq_dst", A("mov r0, 5\nstxdw [r10-8], r0\nlock fetch add [r10-8], r10\n"
                                   "ldxdw r0, [r10-8]\nadd r0, r10\nexit"), r0=5 + 512 + 512,
         cite="emu.rs:433-436,443"),
    Case("q14_cmpxchg_dst_r0", A("mov r3, 7\nstxdw [r10-8], r3\nmov r0, r10\nsub r0, 8\nmov r5, 9\n"
                                 "lock cmpxchg [r0+0], r5\nexit"), r0=504, cite="emu.rs:418,443"),
    # ---- Q15 cmpxchg32 compares the truncated r0 ----
    Case("q15_cmpxchg32", A("mov r3, 7\nstxdw [r10-8], r3\nlddw r0, 0x0000000100000007\nmov r5, 9\n"
                            "lock cmpxchg32 [r10-8], r5\nldxdw r6, [r10-8]\nlsh r6, 8\nor r0, r6\nexit"),
         r0=(9 << 8) | 7, cite="emu.rs:383-386,415"),
    # ---- Q16 only the first byte is bounds-checked (mmu.rs:23-30) ----
    Case("q16_ldxdw_tail_ub", A("ldxdw r0, [r1+1020]\nexit"), status=MEM_UB, cite="mmu.rs:23-30"),
    Case("q16_ldxb_last_ok", A("mov r0, 9\nldxb r0, [r1+1023]\nexit"), r0=0, cite="mmu.rs:23-30"),
    Case("q16_ldxb_past_end", A("ldxb r0, [r1+1024]\nexit"), status=MEM, cite="mmu.rs:26"),
    Case("q16_ldxb_negative", A("ldxb r0, [r1-1]\nexit"), status=MEM, cite="emu.rs:344 as usize"),
    Case("q16_stxw_tail_ub", A("stxw [r1+1022], r1\nexit"), status=MEM_UB, cite="mmu.rs:23-30"),
    Case("q16_stb_last_ok", A("stb [r1+1023], 7\nldxb r0, [r1+1023]\nexit"), r0=7, cite="mmu.rs:23-30"),
    # ---- Q17 register 11 decodes, faults when indexed ----
    Case("q17_r11_unreached", A("mov r0, 3\nexit") + encode(0xB7, 11, 0, 0, 1), r0=3, cite="ins.rs:32"),
    Case("q17_r11_dst", encode(0xB7, 11, 0, 0, 1) + encode(0x95), status=INSN, cite="emu.rs:75"),
    Case("q17_r11_ja_dst", encode(0x05, 11, 0, 0) + encode(0x95), status=INSN, cite="emu.rs:220"),
    Case("q17_r11_ldx_src", encode(0x71, 0, 11, 0) + encode(0x95), status=INSN, cite="emu.rs:320"),
    # ---- Q19 no step limit: a loop runs into the budget ----
    Case("q19_infinite_loop", A("ja -1"), status=STEPS, max_steps=1000, cite="emu.rs:452-458"),
    # ---- Q20 shift counts masked ----
    Case("q20_lsh64_65", A("mov r0, 1\nlsh r0, 65\nexit"), r0=2, cite="emu.rs:115"),
    Case("q20_rsh32_33", A("mov32 r0, 0x80000000\nrsh32 r0, 33\nexit"), r0=0x40000000, cite="emu.rs:120"),
    # ---- Q21 debug-build overflow panics ----
    Case("q21_arsh64_overflow", A("lddw r0, 0x8000000000000000\narsh r0, 64\nexit"), status=ARITH,
         cite="emu.rs:161-162"),
    Case("q21_atomic_add_overflow", A("lddw r3, 0x7FFFFFFFFFFFFFFF\nstxdw [r10-8], r3\nmov r4, 1\n"
                                      "lock add [r10-8], r4\nexit"), status=ARITH, cite="emu.rs:393"),
    Case("q21_atomic32_recombine_overflow", A("lddw r3, 0x7FFFFFFFFFFFFFFF\nstxdw [r10-8], r3\nmov r4, 1\n"
                                              "lock add32 [r10-8], r4\nexit"), status=ARITH,
         cite="emu.rs:427-428"),
    Case("q21_address_overflow", A("lddw r3, 0x7FFFFFFFFFFFFFFF\nldxb r0, [r3+1]\nexit"), status=MEM,
         cite="emu.rs:344"),
    Case("q21_call_ret_overflow", encode(0x85, 0, 0, -2) + encode(0x95), status=ARITH,
         cite="emu.rs:267-268 (pc + 1 on u32)"),
    # ---- Q22 NEG reads regs[src] with the source bit set ----
    Case("q22_neg_src_r11", encode(0x8F, 0, 11, 0) + encode(0x95), status=INSN, cite="emu.rs:68-71"),
    Case("q22_neg_src_ignored", A("mov r0, 5\nmov r3, 9") + encode(0x8F, 0, 3, 0) + encode(0x95),
         r0=(-5) & M64, cite="emu.rs:125"),
    # ---- Q23 initial registers / memory ----
    Case("q23_r10", A("mov r0, r10\nexit"), r0=512, cite="main.rs:31"),
    Case("q23_r1_zero_mem_zero", A("mov r0, r1\nldxdw r3, [r1+100]\nor r0, r3\nexit"), pkt=b"\x01" * 64,
         r0=0, cite="main.rs:16,30"),
    # ---- Q26 JMP32 JA uses off ----
    Case("q26_jmp32_ja", encode(0x06, 0, 0, 1) + A("mov r0, 1\nexit"), r0=0, cite="emu.rs:226-228"),
    # ---- misc: loads/stores through the image ----
    Case("store_packet_then_load", A("stw [r1+2], 0x44332211\nldxdw r0, [r1+0]\nexit"),
         pkt=h("aa bb cc dd ee ff 01 02"), r0=0x020144332211BBAA, cite="emu.rs:361-372"),
    Case("badpkt", A("mov r0, 1\nexit"), pkt=bytes(16), mem_size=8, r10=8, status=BADPKT,
         cite="main.rs:20-21"),
    Case("ld_abs_faults", encode(0x20, 0, 0, 0, 0) + encode(0x95), status=INSN, cite="emu.rs:335-337"),
    Case("ld_mem_faults", encode(0x61 & ~1, 0, 1, 0, 0) + encode(0x95), status=INSN, cite="emu.rs:339"),
    Case("ldx_atomic_mode_faults", encode(0xC1 | 0x18, 0, 1, 0, 0) + encode(0x95), status=INSN,
         cite="emu.rs:351"),
]

# load-time rejects: (name, image, expected error code, expected bad word index, citation)
REJECTS = [
    ("reg12_src", encode(0xB7, 0, 12, 0, 0), -3, 0, "ins.rs:32"),
    ("reg15_dst", encode(0x95) + encode(0xB7, 15, 0, 0, 0), -3, 1, "ins.rs:32"),
    ("alu_op14", encode(0xE7, 0, 0, 0, 0), -4, 0, "ins.rs:251"),
    ("jmp_op15", encode(0x95) + encode(0x95) + encode(0xF5, 0, 0, 0, 0), -4, 2, "ins.rs:257"),
    ("mode_e0", encode(0xE1, 0, 1, 0, 0), -5, 0, "ins.rs:187"),
    ("mode_80_ub", encode(0x81, 0, 1, 0, 0), -5, 0, "ins.rs:188 (invalid discriminant)"),
    ("mode_a0_ub", encode(0xA3, 1, 2, 0, 0), -5, 0, "ins.rs:188 (invalid discriminant)"),
    ("lddw_truncated", encode(0x18, 0, 0, 0, 1), -6, 0, "ins.rs:112"),
    ("lddw_fold_overflow", encode(0x18, 0, 0, 0, -1) + (0x7FFFFFFFFFFFFFFF).to_bytes(8, "little"), -7, 0,
     "ins.rs:112 (debug add overflow)"),
    ("odd_length", encode(0x95)[:5], -2, 0, "ins.rs:66-67"),
    ("invalid_unreachable", encode(0x95) + encode(0xE7), -4, 1, "ins.rs:96-119 (eager decode)"),
]
