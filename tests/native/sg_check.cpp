// Host check of dev/safegcd.h (TEST-ONLY): reads 64-hex-digit integers x (one
// per line, 0 < x < p), prints x^-1 mod p by the 30-bit-limb (argv[1] = "30")
// or 62-bit-limb divsteps, for tests/test_safegcd.py to compare with Python.
#define FTS_HD inline
#include <cstdio>
#include <cstring>

#include "dev/safegcd.h"

int main(int argc, char** argv) {
  const bool s30 = argc > 1 && strcmp(argv[1], "30") == 0;
  char buf[256];
  while (fgets(buf, sizeof buf, stdin)) {
    if (strlen(buf) < 64) continue;
    uint32_t x[8] = {0, 0, 0, 0, 0, 0, 0, 0}, o[8];
    for (int i = 0; i < 64; i++) {
      const char c = buf[i];
      const uint32_t v = c <= '9' ? (uint32_t)(c - '0') : (uint32_t)(c - 'a' + 10);
      const int bit = (63 - i) * 4;
      x[bit / 32] |= v << (bit % 32);
    }
    if (s30)
      fts::sg30_inv_int(x, o);
    else
      fts::sg_inv_int(x, o);
    for (int i = 7; i >= 0; i--) printf("%08x", o[i]);
    printf("\n");
  }
  return 0;
}
