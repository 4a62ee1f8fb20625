// dag_asm.h -- handler numbering of the forward-only micro-op table (host.cpp build_dag stores
// handler_id * DAG_SLOT in DUop::hoff). gen_tile.py reads these ids and emits the tile kernel's
// chained / block-end slots for each (tile_ids.h), and build_tile maps DUop::hoff to them.
#pragma once

#define DAG_SLOT 128

#define H_SLOW 0          // not handled by the asm loop: the C++ step executes it
#define H_EXIT 1
#define H_MOV64_IMM 2     // also LDIMM
#define H_MOV64_REG 3
#define H_ADD64_IMM 4     // also SUB64 imm (negated immediate)
#define H_ADD64_REG 5
#define H_SUB64_REG 6
#define H_AND64_IMM 7
#define H_AND64_REG 8
#define H_OR64_IMM 9
#define H_OR64_REG 10
#define H_XOR64_IMM 11
#define H_XOR64_REG 12
#define H_LSH64_IMM 13
#define H_LSH64_REG 14
#define H_RSH64_IMM 15
#define H_RSH64_REG 16
#define H_MOV32_IMM 17
#define H_MOV32_REG 18
#define H_ADD32_IMM 19    // also SUB32 imm
#define H_ADD32_REG 20
#define H_SUB32_REG 21
#define H_AND32_IMM 22
#define H_AND32_REG 23
#define H_OR32_IMM 24
#define H_OR32_REG 25
#define H_XOR32_IMM 26
#define H_XOR32_REG 27
#define H_LSH32_IMM 28
#define H_LSH32_REG 29
#define H_RSH32_IMM 30
#define H_RSH32_REG 31
#define H_ZX16 32
#define H_ZX32 33
#define H_NOP 34
#define H_BSWAP16 35
#define H_BSWAP32 36
#define H_BSWAP64 37
#define H_JA 38
#define H_JEQ_IMM 39
#define H_JEQ_REG 40
#define H_JGT_IMM 41
#define H_JGT_REG 42
#define H_JLT_IMM 43
#define H_JLT_REG 44
#define H_JSET_IMM 45
#define H_JSET_REG 46
#define H_JEQ32_IMM 47
#define H_JEQ32_REG 48
#define H_JGT32_IMM 49
#define H_JGT32_REG 50
#define H_JLT32_IMM 51
#define H_JLT32_REG 52
#define H_JSET32_IMM 53
#define H_JSET32_REG 54
#define H_LDXK 55         // constant address inside the header window
#define H_LDX 56          // register base: window fast path, anything else bails to C++
// (more kinds; the tile kernel handles every id)
#define H_MUL64_IMM 57
#define H_MUL64_REG 58
#define H_MUL32_IMM 59
#define H_MUL32_REG 60
#define H_NEG64 61
#define H_NEG32 62
#define H_ARSH64_IMM 63
#define H_ARSH64_REG 64
#define H_ARSH32_IMM 65
#define H_ARSH32_REG 66
#define H_DIV64_IMM 67
#define H_DIV64_REG 68
#define H_MOD64_IMM 69
#define H_MOD64_REG 70
#define H_DIV32_IMM 71
#define H_DIV32_REG 72
#define H_MOD32_IMM 73
#define H_MOD32_REG 74
#define H_FAULT 75        // static fault: status in the immediate
#define H_LDXK_FAR 76     // constant address not inside the header window
#define H_COUNT 77
