#!/usr/bin/env python3
"""Generates dag_loop.inc: the hand-written gfx950 interpreter loop of the forward-only fast path
(dag_kernel in interp.hip), as the text of ONE inline-asm statement.

Why asm: the loop is latency-bound per wave (one micro-op per iteration, a chain of SMEM fetch ->
LDS register reads -> dispatch -> commit), and hipcc lowers the C++ switch into a binary compare
tree wrapped in exec-mask flow blocks (~110 instructions per step). Here dispatch is a jump into
fixed 128-byte handler slots (`s_setpc`), exec is narrowed to the lanes parked at the pc, and a
common step is ~25 instructions.

Contract with the C++ side (interp.hip dag_loop_asm):
  in/out  live (SGPR pair): pc set; lpc (VGPR): lane pc; nsteps (VGPR): retired steps
  out     P (SGPR): PC_DONE when no lane is left, else a micro-op the loop does not handle
          (dag_asm.h H_SLOW, or an LDX/LDXK outside the header window or the image): its bit is
          already cleared from live, nothing of it has executed, and the C++ step runs it
  in      prog (DUop table), rl (LDS address of this lane's regs[0]), win (LDS address of this
          lane's header window), swz (its chunk swizzle << 4), len, mem_size
Fixed registers (clobbered): s[64:87] = DUop dwords 0..23 (uop.h), s[88:89] slot base,
s[90:91] the entry exec, s[92:99] and s62 scratch, s63 = min(64, mem_size), v[82:83] A = regs[dst],
v[84:85] S = regs[src], v[86:87] result, v88-v95 scratch, v[96:117] the eBPF register file
(loaded from its LDS home at entry, stored back at exit; indexed with s_set_gpr_idx).
Only plain SALU/VALU/DS/SMEM instructions and VGPR index mode: no VMEM, readlane, DPP, trans or
SDWA, so no gfx950 software wait states are needed inside.

  python3 gen_dag_loop.py > dag_loop.inc
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
IDS = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (H_\w+) (\d+)",
                                                      open(os.path.join(HERE, "dag_asm.h")).read())}
SLOT = 128

# ---- register file: regs[r] of this lane in v[96 + 2r] (low word) and v[97 + 2r] (high word),
#      indexed by s65 = 2 * dst and s66 = 2 * src (s_set_gpr_idx: SRC0 for reads, DST for writes)
READ_A = """s_set_gpr_idx_on s65, gpr_idx(SRC0)
v_mov_b32 v82, v96
v_mov_b32 v83, v97
s_set_gpr_idx_off"""
READ_S = """s_set_gpr_idx_on s66, gpr_idx(SRC0)
v_mov_b32 v84, v96
v_mov_b32 v85, v97
s_set_gpr_idx_off"""


def write(lo, hi):
    return f"""s_set_gpr_idx_on s65, gpr_idx(DST)
v_mov_b32 v96, {lo}
v_mov_b32 v97, {hi}
s_set_gpr_idx_off"""


TAIL_N = """v_mov_b32 %[lpc], s67
v_add_u32 %[nst], 1, %[nst]
s_or_b64 %[live], %[live], s[72:73]
s_branch .Lloop%="""
TAIL_W = write("v86", "v87") + "\n" + TAIL_N
JTAIL = """v_mov_b32 v88, s68
v_mov_b32 v89, s67
v_cndmask_b32 %[lpc], v89, v88, vcc
v_add_u32 %[nst], 1, %[nst]
s_cmp_lg_u64 vcc, 0
s_cselect_b64 s[92:93], s[74:75], 0
s_andn2_b64 s[94:95], exec, vcc
s_cselect_b64 s[94:95], s[72:73], 0
s_or_b64 %[live], %[live], s[92:93]
s_or_b64 %[live], %[live], s[94:95]
s_branch .Lloop%="""


def alu64(op, reg):
    if reg:
        return f"{READ_A}\n{READ_S}\n{op} v86, v84, v82\n{op} v87, v85, v83\n{TAIL_W}"
    return f"{READ_A}\n{op} v86, s76, v82\n{op} v87, s77, v83\n{TAIL_W}"


def alu32(body, reg=False, a=True):
    pre = (READ_A + "\n" if a else "") + (READ_S + "\n" if reg else "")
    return f"{pre}{body}\nv_mov_b32 v87, 0\n{TAIL_W}"


def jump(cmp, reg, pre=""):
    ops = READ_A + "\n" + (READ_S + "\n" if reg else "")
    return f"{ops}{pre}{cmp}\n{JTAIL}"


H = {
    "H_SLOW": """.Lslow%=:
s_mov_b64 exec, s[90:91]
s_mov_b32 %[P], s96
s_branch .Lend%=""",
    "H_EXIT": """v_mov_b32 %[lpc], -1
v_add_u32 %[nst], 1, %[nst]
s_branch .Lloop%=""",
    "H_MOV64_IMM": f"v_mov_b32 v86, s76\nv_mov_b32 v87, s77\n{TAIL_W}",
    "H_MOV64_REG": f"{READ_S}\n{write('v84', 'v85')}\n{TAIL_N}",
    "H_ADD64_IMM": f"{READ_A}\nv_lshl_add_u64 v[86:87], v[82:83], 0, s[76:77]\n{TAIL_W}",
    "H_ADD64_REG": f"{READ_A}\n{READ_S}\nv_lshl_add_u64 v[86:87], v[82:83], 0, v[84:85]\n{TAIL_W}",
    "H_SUB64_REG": f"{READ_A}\n{READ_S}\nv_sub_co_u32 v86, vcc, v82, v84\nv_subb_co_u32 v87, vcc, v83, v85, vcc\n{TAIL_W}",
    "H_AND64_IMM": alu64("v_and_b32", False), "H_AND64_REG": alu64("v_and_b32", True),
    "H_OR64_IMM": alu64("v_or_b32", False), "H_OR64_REG": alu64("v_or_b32", True),
    "H_XOR64_IMM": alu64("v_xor_b32", False), "H_XOR64_REG": alu64("v_xor_b32", True),
    # the hardware uses bits [5:0] / [4:0] of the shift count: the reference's masks (Q20)
    "H_LSH64_IMM": f"{READ_A}\nv_lshlrev_b64 v[86:87], s76, v[82:83]\n{TAIL_W}",
    "H_LSH64_REG": f"{READ_A}\n{READ_S}\nv_lshlrev_b64 v[86:87], v84, v[82:83]\n{TAIL_W}",
    "H_RSH64_IMM": f"{READ_A}\nv_lshrrev_b64 v[86:87], s76, v[82:83]\n{TAIL_W}",
    "H_RSH64_REG": f"{READ_A}\n{READ_S}\nv_lshrrev_b64 v[86:87], v84, v[82:83]\n{TAIL_W}",
    "H_MOV32_IMM": f"v_mov_b32 v86, s76\nv_mov_b32 v87, 0\n{TAIL_W}",
    "H_MOV32_REG": alu32("v_mov_b32 v86, v84", reg=True, a=False),
    "H_ADD32_IMM": alu32("v_add_u32 v86, s76, v82"),
    "H_ADD32_REG": alu32("v_add_u32 v86, v84, v82", reg=True),
    "H_SUB32_REG": alu32("v_sub_u32 v86, v82, v84", reg=True),
    "H_AND32_IMM": alu32("v_and_b32 v86, s76, v82"),
    "H_AND32_REG": alu32("v_and_b32 v86, v84, v82", reg=True),
    "H_OR32_IMM": alu32("v_or_b32 v86, s76, v82"),
    "H_OR32_REG": alu32("v_or_b32 v86, v84, v82", reg=True),
    "H_XOR32_IMM": alu32("v_xor_b32 v86, s76, v82"),
    "H_XOR32_REG": alu32("v_xor_b32 v86, v84, v82", reg=True),
    "H_LSH32_IMM": alu32("v_lshlrev_b32 v86, s76, v82"),
    "H_LSH32_REG": alu32("v_lshlrev_b32 v86, v84, v82", reg=True),
    "H_RSH32_IMM": alu32("v_lshrrev_b32 v86, s76, v82"),
    "H_RSH32_REG": alu32("v_lshrrev_b32 v86, v84, v82", reg=True),
    "H_ZX16": alu32("v_and_b32 v86, 0xffff, v82"),
    "H_ZX32": alu32("v_mov_b32 v86, v82"),
    "H_NOP": TAIL_N,
    # v_perm_b32 selector bytes: 0..3 pick bytes of src1, 0x0c gives 0x00
    "H_BSWAP16": alu32("s_mov_b32 s62, 0x0c0c0001\nv_perm_b32 v86, v82, v82, s62"),
    "H_BSWAP32": alu32("s_mov_b32 s62, 0x00010203\nv_perm_b32 v86, v82, v82, s62"),
    "H_BSWAP64": f"""{READ_A}
s_mov_b32 s62, 0x00010203
v_perm_b32 v86, v83, v83, s62
v_perm_b32 v87, v82, v82, s62
{TAIL_W}""",
    "H_JA": """v_mov_b32 %[lpc], s68
v_add_u32 %[nst], 1, %[nst]
s_or_b64 %[live], %[live], s[74:75]
s_branch .Lloop%=""",
    # jumps: vcc = condition over the active lanes; x / npc, tbit / nbit already canonical
    "H_JEQ_IMM": jump("v_cmp_eq_u64 vcc, s[76:77], v[82:83]", False),
    "H_JEQ_REG": jump("v_cmp_eq_u64 vcc, v[84:85], v[82:83]", True),
    "H_JGT_IMM": jump("v_cmp_lt_i64 vcc, s[76:77], v[82:83]", False),   # k < A
    "H_JGT_REG": jump("v_cmp_lt_i64 vcc, v[84:85], v[82:83]", True),
    "H_JLT_IMM": jump("v_cmp_gt_i64 vcc, s[76:77], v[82:83]", False),   # k > A
    "H_JLT_REG": jump("v_cmp_gt_i64 vcc, v[84:85], v[82:83]", True),
    "H_JSET_IMM": f"""{READ_A}
v_and_b32 v88, s76, v82
v_and_b32 v89, s77, v83
v_or_b32 v88, v88, v89
v_cmp_ne_u32 vcc, 0, v88
s_branch .Ljtail%=""",
    "H_JSET_REG": f"""{READ_A}
{READ_S}
v_and_b32 v88, v84, v82
v_and_b32 v89, v85, v83
v_or_b32 v88, v88, v89
v_cmp_ne_u32 vcc, 0, v88
s_branch .Ljtail%=""",
    # JMP32: signed compares of the low words == compares of the sign-extended words (Q3)
    "H_JEQ32_IMM": jump("v_cmp_eq_u32 vcc, s76, v82", False),
    "H_JEQ32_REG": jump("v_cmp_eq_u32 vcc, v84, v82", True),
    "H_JGT32_IMM": jump("v_cmp_lt_i32 vcc, s76, v82", False),
    "H_JGT32_REG": jump("v_cmp_lt_i32 vcc, v84, v82", True),
    "H_JLT32_IMM": jump("v_cmp_gt_i32 vcc, s76, v82", False),
    "H_JLT32_REG": jump("v_cmp_gt_i32 vcc, v84, v82", True),
    "H_JSET32_IMM": jump("v_cmp_ne_u32 vcc, 0, v88", False, "v_and_b32 v88, s76, v82\n"),
    "H_JSET32_REG": jump("v_cmp_ne_u32 vcc, 0, v88", True, "v_and_b32 v88, v84, v82\n"),
    "H_LDXK": "s_branch .Lldxk%=",
    "H_LDX": "s_branch .Lldx%=",
}

WAIT = "s_waitcnt lgkmcnt(0)"


# Shared tail of a window load: v88..v90 = the three window dwords (in flight), byte shift in
# SHIFT, a0 in A0 (SGPR or VGPR); mask to the access width (s[70:71]), zero the bytes at or past
# len, merge into the old dst value (Q1) and commit.
def window_tail(a0, shift):
    return f"""v_sub_u32 v94, %[len], {a0}
v_cmp_lt_u32 vcc, {a0}, %[len]
v_cndmask_b32 v94, 0, v94, vcc
v_min_u32 v94, 8, v94
v_lshlrev_b32 v94, 3, v94
v_sub_u32 v94, 64, v94
{READ_A}
{WAIT}
v_alignbyte_b32 v86, v89, v88, {shift}
v_alignbyte_b32 v87, v90, v89, {shift}
v_and_b32 v86, s70, v86
v_and_b32 v87, s71, v87
v_lshlrev_b64 v[86:87], v94, v[86:87]
v_lshrrev_b64 v[86:87], v94, v[86:87]
v_cndmask_b32 v86, 0, v86, vcc
v_cndmask_b32 v87, 0, v87, vcc
v_bfi_b32 v86, s70, v86, v82
v_bfi_b32 v87, s71, v87, v83
{TAIL_W}"""


# LDXK: constant address a0 = s69, end = s79 (<= 64 by construction), window dword i at chunk
# bits s[80 + 2i] (xor'ed with the lane swizzle), byte-in-chunk s[81 + 2i]
LDXK = """.Lldxk%=:
s_cmp_gt_u32 s79, %[mem]
s_cbranch_scc1 .Lslow%=
v_xor_b32 v88, s80, %[swz]
v_add3_u32 v88, %[win], v88, s81
v_xor_b32 v89, s82, %[swz]
v_add3_u32 v89, %[win], v89, s83
v_xor_b32 v90, s84, %[swz]
v_add3_u32 v90, %[win], v90, s85
ds_read_b32 v88, v88
ds_read_b32 v89, v89
ds_read_b32 v90, v90
s_and_b32 s62, s69, 3
""" + window_tail("s69", "s62")

# LDX: address = S + sext(off) (s[76:77]); every active lane must land in the window and the image
# (high word 0 -- which also excludes a signed overflow -- and addr + width <= min(64, mem_size)),
# else the C++ step runs it (faults, reads past the window)
LDX = f""".Lldx%=:
{READ_S}
v_lshl_add_u64 v[92:93], v[84:85], 0, s[76:77]
v_add_u32 v94, s78, v92
v_cmp_ne_u32_e64 s[92:93], 0, v93
v_cmp_gt_u32_e64 s[94:95], v94, s63
s_or_b64 s[92:93], s[92:93], s[94:95]
s_cbranch_scc1 .Lslow%=
v_and_b32 v93, -4, v92
v_and_b32 v88, 48, v93
v_xor_b32 v88, v88, %[swz]
v_and_b32 v95, 15, v93
v_add3_u32 v88, %[win], v88, v95
v_add_u32 v89, 4, v93
v_min_u32 v89, 60, v89
v_and_b32 v95, 48, v89
v_xor_b32 v95, v95, %[swz]
v_and_b32 v89, 15, v89
v_add3_u32 v89, %[win], v95, v89
v_add_u32 v90, 8, v93
v_min_u32 v90, 60, v90
v_and_b32 v95, 48, v90
v_xor_b32 v95, v95, %[swz]
v_and_b32 v90, 15, v90
v_add3_u32 v90, %[win], v95, v90
ds_read_b32 v88, v88
ds_read_b32 v89, v89
ds_read_b32 v90, v90
v_and_b32 v93, 3, v92
""" + window_tail("v92", "v93")

# the LDS home of the register file (interp.hip's [11][64] u64 layout, 512 B per register)
LOAD_REGS = "\n".join(f"ds_read_b64 v[{96 + 2 * r}:{97 + 2 * r}], %[rl] offset:{512 * r}"
                      for r in range(11)) + "\n" + WAIT
STORE_REGS = "\n".join(f"ds_write_b64 %[rl], v[{96 + 2 * r}:{97 + 2 * r}] offset:{512 * r}"
                       for r in range(11)) + "\n" + WAIT

PROLOGUE = LOAD_REGS + """
s_mov_b64 s[90:91], exec
s_min_u32 s63, %[mem], 64
s_getpc_b64 s[88:89]
.Lpc%=:
s_add_u32 s88, s88, .Lslots%=-.Lpc%=
s_addc_u32 s89, s89, 0
.Lloop%=:
s_mov_b64 exec, s[90:91]
s_ff1_i32_b64 s96, %[live]
s_cmp_lt_i32 s96, 0
s_cbranch_scc1 .Ldone%=
s_bitset0_b64 %[live], s96
s_lshl_b32 s97, s96, 8
s_load_dwordx16 s[64:79], %[prog], s97
s_add_u32 s97, s97, 64
s_load_dwordx8 s[80:87], %[prog], s97
v_cmp_eq_u32 vcc, s96, %[lpc]
s_mov_b64 exec, vcc
s_waitcnt lgkmcnt(0)
s_add_u32 s98, s88, s64
s_addc_u32 s99, s89, 0
s_setpc_b64 s[98:99]
.Ljtail%=:
""" + JTAIL + """
.p2align 7
.Lslots%=:"""

EPILOGUE = """.Ldone%=:
s_mov_b32 %[P], -1
.Lend%=:
""" + STORE_REGS


def main():
    order = sorted(IDS.items(), key=lambda kv: kv[1])
    names = [n for n, i in order if n != "H_COUNT"]
    assert [IDS[n] for n in names] == list(range(len(names))), "handler ids must be dense"
    parts = [PROLOGUE]
    for n in names:  # ids this loop does not implement go to the C++ step
        parts.append(f"; {n}\n.org .Lslots%=+{IDS[n] * SLOT}\n" + H.get(n, "s_branch .Lslow%="))
    parts.append(f".org .Lslots%=+{IDS['H_COUNT'] * SLOT}")
    parts += [LDXK, LDX, EPILOGUE]
    text = "\n".join(parts)
    out = ["// GENERATED by gen_dag_loop.py from dag_asm.h -- do not edit. One inline-asm statement.",
           "// clang-format off"]
    for line in text.splitlines():
        out.append('"' + line.replace("\\", "\\\\").replace('"', '\\"') + '\\n"')
    out.append("// clang-format on")
    print("\n".join(out))


if __name__ == "__main__":
    main()
