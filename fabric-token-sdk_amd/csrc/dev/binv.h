// Montgomery's batch inversion over one 256-lane workgroup (device only): each
// lane hands in an Fp value, a product tree in LDS multiplies them up to the
// root, one variable-time binary Euclid (fp_inv_var) inverts the root, and the
// inverses are handed down the tree (inv(a) = inv(ab) b, inv(b) = inv(ab) a).
// A zero input is replaced by 1 for the tree and comes back as 0.  Every value
// inverted on these paths is public (a verification batch's norms), so the
// variable-time Euclid is allowed, as in f2_inv_inl.
//
// Used where one inversion per job was the larger part of a launch's
// instructions (k_fexp_binv: the easy part's norms; k_g2_binv: the norms of
// t''s Z before the line chain).
#pragma once
#include "fp.h"

namespace fts {

#ifndef FTS_BINV_PRIO
#define FTS_BINV_PRIO 3  // wave priority of a tree launch: its lone Euclid shares a SIMD with other slots' waves
#endif

// t = threadIdx.x (blockDim 256); get() is called only when active, put(v)
// likewise; tree: 512 x 8 words of LDS (heap order: root 1, node i's children
// 2i and 2i + 1, leaves 256..511)
template <class Get, class Put>
__device__ __forceinline__ void binv_tree256(uint32_t (*tree)[8], uint32_t t, bool active, const Get& get,
                                             const Put& put) {
  __builtin_amdgcn_s_setprio(FTS_BINV_PRIO);
  fp v = fe_one<ModP>();
  bool zero = false;
  if (active) {
    v = get();
    zero = fe_is_zero(v);
    if (zero) v = fe_one<ModP>();
  }
  auto st = [&](uint32_t i, const fp& a) {
#pragma unroll
    for (int q = 0; q < 8; q++) tree[i][q] = a.v[q];
  };
  auto ld = [&](uint32_t i) {
    fp a;
#pragma unroll
    for (int q = 0; q < 8; q++) a.v[q] = tree[i][q];
    return a;
  };
  st(256 + t, v);
  __syncthreads();
  for (uint32_t w = 128; w >= 1; w >>= 1) {
    if (t < w) st(w + t, ld(2 * (w + t)) * ld(2 * (w + t) + 1));
    __syncthreads();
  }
  if (t == 0) st(1, fp_inv_var(ld(1)));
  __syncthreads();
  for (uint32_t w = 1; w <= 128; w <<= 1) {
    fp ia, ib;
    if (t < w) {
      const uint32_t p = w + t;
      const fp ip = ld(p), a = ld(2 * p), b = ld(2 * p + 1);
      ia = ip * b;
      ib = ip * a;
    }
    __syncthreads();
    if (t < w) {
      st(2 * (w + t), ia);
      st(2 * (w + t) + 1, ib);
    }
    __syncthreads();
  }
  if (active) put(zero ? fe_zero<ModP>() : ld(256 + t));
}

}  // namespace fts
