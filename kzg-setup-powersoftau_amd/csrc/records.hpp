// Record I/O shared by the kernels: 48-B coordinates as 12 x 32-bit words, big-endian (pairing)
// or little-endian (ark) on the wire; status reporting; the opaque-pointer reload idiom.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fp381.hpp"

namespace kzgpot {

KZG_DEV uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

KZG_DEV void report(uint64_t i, int st, unsigned long long* first_bad, uint8_t* status) {
  if (status) status[i] = (uint8_t)st;
  if (st) atomicMin(first_bad, (unsigned long long)((i << 8) | (uint64_t)st));
}

// Hide a pointer from the optimiser so loads through it are re-issued at every use (keeps the
// affine base point and the raw input words out of the register file during the long chains).
template <typename T>
KZG_DEV const T* opaque(const T* p) {
  asm volatile("" : "+v"(p));
  return p;
}

// ---------------------------------------------------------------- 48-B coordinates <-> words
// A coordinate travels as 12 little-endian 32-bit words (the 384-bit integer); fp381.hpp converts
// words <-> 14 x 28-bit limbs. Flag bits live in word 11 (bits 381..383).
using words = uint32_t[12];

KZG_DEV void load_le(words& w, const uint4* src) {  // 48 little-endian bytes (ark)
  const uint4 a = src[0], b = src[1], c = src[2];
  w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w;
  w[4] = b.x, w[5] = b.y, w[6] = b.z, w[7] = b.w;
  w[8] = c.x, w[9] = c.y, w[10] = c.z, w[11] = c.w;
}
KZG_DEV void load_be(words& w, const uint4* src) {  // 48 big-endian bytes (pairing)
  const uint4 a = src[0], b = src[1], c = src[2];
  const uint32_t r[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
  for (int k = 0; k < 12; k++) w[k] = bswap32(r[11 - k]);
}
KZG_DEV void store_words(uint4* dst, const words& w) {
  dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
  dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
  dst[2] = make_uint4(w[8], w[9], w[10], w[11]);
}
KZG_DEV void store_canon(uint4* dst, const fp& c) {  // canonical element -> 48 LE bytes
  words w;
  fp_to_words(w, c);
  store_words(dst, w);
}
KZG_DEV void store_zero(uint4* dst, int n16) {
#pragma unroll 1
  for (int k = 0; k < n16; k++) dst[k] = make_uint4(0, 0, 0, 0);
}
KZG_DEV void zero_words(words& w) {
#pragma unroll
  for (int k = 0; k < 12; k++) w[k] = 0;
}
// canonical words -> Montgomery element (reduced: value < 1.002 p)
KZG_DEV void words_to_mont(fp& r, const words& w) {
  fp t;
  fp_from_words(t, w);
  fp_to_mont(r, t);
}

}  // namespace kzgpot
