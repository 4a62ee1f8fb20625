/*
 * ebpf_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference interpreter b1tg/ebpf-emu (snapshot 2024-12-20):
 *   decode   : src/ins.rs:96-173 (+ enum ranges ins.rs:13-35,175-279)
 *   execute  : src/emu.rs:48-458
 *   memory   : src/mmu.rs:7-30
 *   layout   : src/main.rs:14-43
 *
 * This oracle is the CHECKER for the HIP product path. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product library (libebpfemu.so) never
 * links it and never falls back to it.
 *
 * Parity pinning: the reference is Rust and no Rust toolchain exists in this environment, so
 * it cannot be executed here. The oracle is pinned by (a) the reference's own decode unit
 * tests (ins.rs:291-500), (b) the three program KATs embedded in the reference (ins.rs:435,
 * notes.md:27, Makefile:16) and the behaviours its comments quote from bpf_conformance
 * (emu.rs:97,108-111,131,150-155; main.rs:26-28), and (c) an independently written Python
 * restatement (oracle/pyref.py) cross-checked by differential fuzzing. The 180-vector
 * bpf_conformance suite (notes.md:19) is absent (empty submodule): that part is UNPINNED.
 *
 * Where the reference panics (a Rust debug build, as its CI and Makefile run it:
 * build.yml:29,40, Makefile:8) the oracle returns a fault status instead of r0. Where the
 * reference hangs (no step limit, emu.rs:452-458) or has undefined behaviour (mmu.rs:23-30
 * tail bytes; ins.rs:188 invalid Mode discriminants 0x80/0xa0) the oracle defines a status.
 */
#ifndef EBPF_ORACLE_H
#define EBPF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Decoded instruction, field-for-field ins.rs:37-45 (`code` kept as the raw opcode byte). */
typedef struct or_insn {
  int32_t imm;
  int64_t imm64;
  int16_t off;
  uint8_t src;
  uint8_t dst;
  uint8_t code;
} or_insn;

/* Load-time rejects (the reference panics while decoding, ins.rs). Same numbering as
 * include/ebpf_emu.h EBPF_E*. */
#define OR_E_LEN      (-2)  /* nbytes % 8 != 0: hexs_to_u64s "invalid hex format for u64" ins.rs:66-67 */
#define OR_E_REG      (-3)  /* register nibble >= 12: assert ins.rs:32 */
#define OR_E_OP       (-4)  /* ALU/JMP op nibble > 0xd: assert ins.rs:251,257 */
#define OR_E_MODE     (-5)  /* LS mode 0xe0 (assert ins.rs:187) or 0x80/0xa0 (invalid discriminant, UB) */
#define OR_E_LDDW     (-6)  /* wide insn without a second word: index panic ins.rs:112 */
#define OR_E_LDDW_OVF (-7)  /* imm64 fold overflows i64 (debug-build panic, ins.rs:112) */

/* Per-execution status codes. Same numbering as include/ebpf_emu.h EBPF_ST_*. */
#define OR_ST_OK        0  /* exit with empty frame stack (emu.rs:277) or pc past the end (emu.rs:49,448) */
#define OR_ST_MEM       1  /* memory bounds panic (mmu.rs:16,26) or address overflow (emu.rs:344,367,375) */
#define OR_ST_MEM_UB    2  /* first byte in bounds, tail out of bounds: UB in the reference (mmu.rs:23-30) */
#define OR_ST_INSN      3  /* runtime panic on an instruction: reg 11 indexed, END imm, callx, ABS/IND,
                              LD+MEM, bad mode for class, unknown atomic op (emu.rs:206,270,336,339,351,421,438) */
#define OR_ST_ARITH     4  /* debug overflow panic: arsh64 (emu.rs:162), atomic add (emu.rs:393,427),
                              call return address (emu.rs:268) */
#define OR_ST_STEPS     5  /* step budget exhausted (the reference has none and hangs, emu.rs:452) */
#define OR_ST_CALLDEPTH 6  /* frame stack deeper than OR_MAX_CALL_DEPTH (reference: unbounded Vec) */
#define OR_ST_BADPKT    7  /* packet longer than the memory image (main.rs:20-21 index panic) */

#define OR_MAX_CALL_DEPTH 64

/* Decode a little-endian program image (the byte sequence the reference's hex encodes;
 * hexs_to_u64s + from_be, ins.rs:60-74,97). Returns the number of decoded instructions
 * (>= 0) or an OR_E_* code; *bad_word receives the index of the offending 8-byte word. */
long or_decode(const uint8_t* code, size_t nbytes, or_insn* out, size_t cap, size_t* bad_word);

/* Run one execution (Emu::run, emu.rs:452-458) on a caller-owned memory image and register
 * file. max_steps == 0 means unlimited. *steps receives the number of instructions
 * executed (the final exit included, a faulting instruction excluded). Returns OR_ST_*. */
int or_run(const or_insn* prog, size_t n, uint8_t* mem, size_t mem_size, int64_t regs[11],
           uint64_t max_steps, uint64_t* steps);

/* or_run with the frame stack exposed (Emu.fp is pub, emu.rs:26): fp[0..*fp_len) is the initial
 * stack (bottom first; an EXIT pops its top, emu.rs:273-279), and on return the final stack. */
int or_run_fp(const or_insn* prog, size_t n, uint8_t* mem, size_t mem_size, int64_t regs[11],
              uint32_t fp[OR_MAX_CALL_DEPTH], size_t* fp_len, uint64_t max_steps,
              uint64_t* steps);

/* One packet with the reference harness layout (main.rs:14-31): zeroed mem_size image,
 * packet copied to [0,len), r1 = 0, r2 = len, r10 = r10_init, other registers 0. */
int or_run_packet(const or_insn* prog, size_t n, const uint8_t* pkt, size_t len, size_t mem_size,
                  uint64_t r10_init, uint64_t max_steps, uint64_t* r0, uint64_t* steps);

/* Batch over a frame buffer (stride layout when offsets == NULL; len = lens[i] or stride),
 * split over `threads` host threads with static contiguous partitions. Outputs may be NULL.
 * counters[8]: [0..4] r0 == 0..4 (xdp_action, xdp.rs:3-9), [5] other r0, [6] faults,
 * [7] instructions retired. Returns 0. */
int or_run_batch(const or_insn* prog, size_t n, const uint8_t* frames, const uint32_t* offsets,
                 const uint16_t* lens, uint64_t stride, uint64_t npkts, size_t mem_size,
                 uint64_t r10_init, uint64_t max_steps, uint64_t* r0_out, uint8_t* status_out,
                 uint64_t counters[8], int threads);
/* The same with xdp != 0: each packet runs as the xdp_md image [u32 data = 8][u32 data_end =
 * 8 + len][packet] (xdp.rs:16-20) handed to main.rs (r2 = 8 + len, main.rs:18-29). */
int or_run_batch_xdp(const or_insn* prog, size_t n, const uint8_t* frames,
                     const uint32_t* offsets, const uint16_t* lens, uint64_t stride, uint64_t npkts,
                     size_t mem_size, uint64_t r10_init, uint64_t max_steps, uint64_t* r0_out,
                     uint8_t* status_out, uint64_t counters[8], int threads, int xdp);

#ifdef __cplusplus
}
#endif
#endif
