// Loader mirror: ark-ec 0.2 `GroupAffine::deserialize_unchecked` over a
// kgz / fastkzg setup file — the per-point work of `load_kzg_setup` / `load_fastkzg_setup`
// (src/lib.rs:174-228). Per point:
//   x  = Fp::deserialize        (48 B LE, x < p else InvalidData)
//   y  = Fp::deserialize_with_flags::<SWFlags> (flags = top 2 bits of the last byte; both set ->
//        UnexpectedFlags; masked y < p else InvalidData)
//   GroupAffine::new(x, y, infinity)            — no curve check, no subgroup check ("unchecked")
// G2: x = (c0, c1), y = (c0, c1 with the flags), each component as above.
//
// Output: the in-memory arkworks layout a Rust caller transmutes into `GroupAffine<P>` — ark-ff
// Montgomery form (R = 2^384) as 6 little-endian u64 per Fp, then the `infinity` bool and
// padding to 8 B: G1 104 B (x 48 | y 48 | inf 1 | pad 7), G2 200 B (x.c0 | x.c1 | y.c0 | y.c1 |
// inf | pad). Rejected points are zero-filled.
//
// HBM-bound: 96 B in + 104 B out per G1 point against 2 Fp multiplies.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec.hpp"
#include "fp381.hpp"
#include "records.hpp"

namespace kzgpot {

// canonical words (< p) -> ark Montgomery words: x 2^384 mod p
KZG_DEV void words_to_ark_mont(words& out, const words& w) {
  fp x, k;
  fp_from_words(x, w);
  fp_set(k, FP_ARK_R);
  fp_mul(x, x, k);
  fp_reduce_canon(x, x);
  fp_to_words(out, x);
}

KZG_DEV void store_u64x(uint2* dst, const words& w) {  // 48 B at an 8-B aligned address
#pragma unroll
  for (int k = 0; k < 6; k++) dst[k] = make_uint2(w[2 * k], w[2 * k + 1]);
}

__global__ void __launch_bounds__(kBlock) k_g1_load(const uint4* __restrict__ in, uint2* __restrict__ out,
                                                    uint64_t n, unsigned long long* __restrict__ first_bad,
                                                    uint8_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  words x, y;
  load_le(x, in + i * 6);
  load_le(y, in + i * 6 + 3);
  const uint32_t yb = y[11] >> 24;
  const bool fpos = yb & 0x80u, finf = yb & 0x40u;
  y[11] &= 0x3fffffffu;
  int st = 0;
  if (words_geq_p(x)) st = 3;
  else if (fpos && finf) st = 6;
  else if (words_geq_p(y)) st = 3;
  uint2* dst = out + i * 13;
  if (st) {
#pragma unroll
    for (int k = 0; k < 13; k++) dst[k] = make_uint2(0, 0);
  } else {
    words m;
    words_to_ark_mont(m, x);
    store_u64x(dst, m);
    words_to_ark_mont(m, y);
    store_u64x(dst + 6, m);
    dst[12] = make_uint2(finf ? 1u : 0u, 0u);
  }
  report(i, st, first_bad, status);
}

__global__ void __launch_bounds__(kBlock) k_g2_load(const uint4* __restrict__ in, uint2* __restrict__ out,
                                                    uint64_t n, unsigned long long* __restrict__ first_bad,
                                                    uint8_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint4* rec = in + i * 12;
  int st = 0;
  bool finf;
  {
    words c;
    load_le(c, rec + 9);  // y.c1 carries the flags
    const uint32_t yb = c[11] >> 24;
    const bool fpos = yb & 0x80u;
    finf = yb & 0x40u;
    c[11] &= 0x3fffffffu;
    words a;
    load_le(a, rec);
    if (words_geq_p(a)) st = 3;
    load_le(a, rec + 3);
    if (!st && words_geq_p(a)) st = 3;
    load_le(a, rec + 6);
    if (!st && words_geq_p(a)) st = 3;
    if (!st && fpos && finf) st = 6;
    if (!st && words_geq_p(c)) st = 3;
  }
  uint2* dst = out + i * 25;
  if (st) {
#pragma unroll 1
    for (int k = 0; k < 25; k++) dst[k] = make_uint2(0, 0);
  } else {
#pragma unroll 1
    for (int c = 0; c < 4; c++) {
      words w, m;
      load_le(w, rec + 3 * c);
      if (c == 3) w[11] &= 0x3fffffffu;
      words_to_ark_mont(m, w);
      store_u64x(dst + 6 * c, m);
    }
    dst[24] = make_uint2(finf ? 1u : 0u, 0u);
  }
  report(i, st, first_bad, status);
}

hipError_t launch_load(bool g2, const void* d_in, void* d_out, uint64_t n, unsigned long long* d_first_bad,
                       uint8_t* d_status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock)), block(kBlock);
  if (g2)
    hipLaunchKernelGGL(k_g2_load, grid, block, 0, stream, (const uint4*)d_in, (uint2*)d_out, n, d_first_bad,
                       d_status);
  else
    hipLaunchKernelGGL(k_g1_load, grid, block, 0, stream, (const uint4*)d_in, (uint2*)d_out, n, d_first_bad,
                       d_status);
  return hipGetLastError();
}

}  // namespace kzgpot
