/* fuzz_main.c — TEST INFRASTRUCTURE ONLY: drives the oracle over random programs and packets so
 * that an -fsanitize=address,undefined build can check it for memory errors / UB. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ebpf_oracle.h"

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { /* splitmix64 */
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static const uint8_t OPS[] = {0x07, 0x0f, 0x17, 0x1f, 0x27, 0x2f, 0x37, 0x3f, 0x47, 0x4f, 0x57, 0x5f,
                              0x67, 0x6f, 0x77, 0x7f, 0x87, 0x97, 0x9f, 0xa7, 0xaf, 0xb7, 0xbf, 0xc7,
                              0xcf, 0xd4, 0xdc, 0x04, 0x0c, 0x14, 0x34, 0x3c, 0x64, 0x74, 0x84, 0x94,
                              0xa4, 0xb4, 0xbc, 0xc4, 0x05, 0x15, 0x1d, 0x25, 0x2d, 0x35, 0x45, 0x55,
                              0x65, 0x75, 0xa5, 0xb5, 0xc5, 0xd5, 0x16, 0x26, 0x06, 0x85, 0x95, 0x95,
                              0x61, 0x69, 0x71, 0x79, 0x62, 0x6a, 0x72, 0x7a, 0x63, 0x6b, 0x73, 0x7b,
                              0xc3, 0xdb, 0x18, 0x20, 0x8d, 0xe7, 0x81};

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 20000;
  uint8_t img[8 * 48];
  or_insn prog[48];
  uint8_t pkt[128];
  size_t hist[9] = {0};
  for (int it = 0; it < iters; it++) {
    int nw = 1 + (int)(rnd() % 40);
    for (int i = 0; i < nw; i++) {
      uint64_t w = rnd();
      uint8_t op = OPS[rnd() % sizeof OPS];
      uint8_t regs = (uint8_t)((rnd() % 12) | ((rnd() % 12) << 4));
      int16_t off = (int16_t)((rnd() % 4) ? (int)(rnd() % 80) - 8 : (int)(rnd() % 2048) - 1024);
      memcpy(img + 8 * i, &op, 1);
      memcpy(img + 8 * i + 1, &regs, 1);
      memcpy(img + 8 * i + 2, &off, 2);
      memcpy(img + 8 * i + 4, (uint8_t*)&w + 4, 4);
    }
    size_t bad = 0;
    long n = or_decode(img, 8 * (size_t)nw, prog, 48, &bad);
    if (n < 0) { hist[8]++; continue; }
    size_t len = (size_t)(rnd() % 100);
    for (size_t i = 0; i < len; i++) pkt[i] = (uint8_t)rnd();
    uint64_t r0 = 0, steps = 0;
    int st = or_run_packet(prog, (size_t)n, pkt, len, 1024, 512, 500, &r0, &steps);
    hist[st & 7]++;
  }
  printf("status histogram:");
  for (int i = 0; i < 9; i++) printf(" %zu", hist[i]);
  printf("\n");
  return 0;
}
