// SHA-256 (FIPS 180-4) per lane, streamed over byte segments of a device arena.
// Replaces crypto/sha256 inside mathlib HashToZr.
#pragma once
#include "fp.h"

namespace fts {

// Round constants: a __constant__ array for the device; the host build (the
// test emulation, and host code of the product library such as the native
// Setup, host/setup.cpp) reads its own copy -- in a HIP compile the host side
// of a __constant__ variable is only a shadow and must not be read.
#define FTS_SHA_K_VALUES \
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,  \
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,  \
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,  \
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,  \
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,  \
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,  \
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,  \
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u
#ifdef __HIPCC__
__device__ __constant__ static const uint32_t SHA_K_D[64] = {FTS_SHA_K_VALUES};
#endif
static const uint32_t SHA_K_H[64] = {FTS_SHA_K_VALUES};
#if defined(__HIP_DEVICE_COMPILE__)
#define SHA_K SHA_K_D
#else
#define SHA_K SHA_K_H
#endif

FTS_HD uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct Sha256 {
  uint32_t h[8];
  uint32_t w[16];  // current block as big-endian words
  uint32_t fill;   // bytes in current block
  uint64_t total;

  FTS_HD void init() {
    h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
    h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
    fill = 0;
    total = 0;
    for (int i = 0; i < 16; i++) w[i] = 0;
  }

  // one 64-byte block given as 16 big-endian words (fully unrolled: the
  // message schedule stays in registers)
  FTS_HD void compress_words(const uint32_t* in) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; i++) W[i] = in[i];
#pragma unroll
    for (int i = 0; i < 64; i++) {
      uint32_t wi;
      if (i < 16) {
        wi = W[i];
      } else {
        uint32_t w15 = W[(i - 15) & 15], w2 = W[(i - 2) & 15];
        uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
        uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
        wi = W[i & 15] + s0 + W[(i - 7) & 15] + s1;
        W[i & 15] = wi;
      }
      uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
      uint32_t ch = (e & f) ^ (~e & g);
      uint32_t t1 = hh + S1 + ch + SHA_K[i] + wi;
      uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
      uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }

  FTS_HD void compress() {
    compress_words(w);
    for (int i = 0; i < 16; i++) w[i] = 0;
    fill = 0;
  }

  FTS_HD void byte(uint8_t x) {
    w[fill >> 2] |= (uint32_t)x << (24 - 8 * (fill & 3));
    fill++;
    total++;
    if (fill == 64) compress();
  }

  FTS_HD void update(const uint8_t* p, uint32_t n) {
    uint32_t i = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    // whole blocks straight from memory with 16-byte loads while the block is
    // empty and the source 16-byte aligned (the planners align every arena
    // allocation to 16 bytes; transcript segments are 64-byte multiples except
    // the last)
    if (fill == 0 && (((uintptr_t)p) & 15) == 0) {
      while (n - i >= 64) {
        const uint4* q = reinterpret_cast<const uint4*>(p + i);
        uint32_t W[16];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          uint4 v = q[k];
          W[4 * k] = __builtin_bswap32(v.x);
          W[4 * k + 1] = __builtin_bswap32(v.y);
          W[4 * k + 2] = __builtin_bswap32(v.z);
          W[4 * k + 3] = __builtin_bswap32(v.w);
        }
        compress_words(W);
        total += 64;
        i += 64;
      }
    }
#endif
    // whole words when the block position is word-aligned
    while (i < n && (fill & 3)) byte(p[i++]);
    while (i + 4 <= n) {
      w[fill >> 2] = ((uint32_t)p[i] << 24) | ((uint32_t)p[i + 1] << 16) | ((uint32_t)p[i + 2] << 8) | p[i + 3];
      fill += 4;
      total += 4;
      i += 4;
      if (fill == 64) compress();
    }
    while (i < n) byte(p[i++]);
  }

  FTS_HD void final(uint8_t out[32]) {
    uint64_t bits = total * 8;
    byte(0x80);
    total--;  // padding bytes do not count
    while (fill != 56) {
      byte(0);
      total--;
    }
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    compress();
    for (int i = 0; i < 8; i++) {
      out[4 * i] = (uint8_t)(h[i] >> 24);
      out[4 * i + 1] = (uint8_t)(h[i] >> 16);
      out[4 * i + 2] = (uint8_t)(h[i] >> 8);
      out[4 * i + 3] = (uint8_t)h[i];
    }
  }
};

// HashToZr: SHA-256 digest read big-endian, reduced mod r (limbs, canonical)
FTS_HD void digest_mod_r(uint32_t out[8], const uint8_t d[32]) {
  uint32_t x[8];
  be32_to_limbs(x, d);
  uint32_t mm[8];
  for (int i = 0; i < 8; i++) mm[i] = R_MOD[i];
  for (int k = 0; k < 6; k++) {
    uint32_t t[8];
    uint32_t br = sub8(t, x, mm);
    if (!br)
      for (int i = 0; i < 8; i++) x[i] = t[i];
  }
  for (int i = 0; i < 8; i++) out[i] = x[i];
}

}  // namespace fts
