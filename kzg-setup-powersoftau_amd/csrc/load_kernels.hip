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
// HBM-bound: 96 B in + 104 B out per G1 point against 2 Fp multiplies; global traffic is staged
// through LDS so that it is fully coalesced.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec.hpp"
#include "fp381.hpp"
#include "records.hpp"

namespace kzgpot {

// canonical words (< p) -> ark Montgomery words: x 2^384 mod p, a multiplication by a CONSTANT,
// so the reduction is folded into precomputed constants instead of a full Montgomery multiply:
//   S = sum_k x_k C_k,  C_k = 2^(384 + 56 + 32 k) mod p  (FP_ARK_WORD: the 12 input words times
//       14-limb constants — 168 single-mad columns, each < 12 x 2^32 x 2^28 < 2^63.6),
//   then two Montgomery digit steps divide by 2^56: (S + m0 p + m1 p 2^28) / 2^56 = x 2^384
//   (mod p), and S < 12 x 2^32 p makes it < 1.000001 p, so one conditional subtraction finishes.
// 196 product mads and no word <-> limb conversion of the input, against fp_from_words + a
// 392-mad fp_mul by 2^384 R. Any 384-bit input keeps every bound (the caller rejects x >= p).
KZG_DEV void words_to_ark_mont(words& out, const words& w) {
  constexpr int N = BlsFp::NL;
  uint64_t col[N + 1];
#pragma unroll
  for (int j = 0; j < N; j++) {
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) acc += (uint64_t)w[k] * FP_ARK_WORD[k][j];
    col[j] = acc;
  }
  col[N] = 0;
#pragma unroll
  for (int s = 0; s < 2; s++) {  // col[s] becomes a multiple of 2^28 and its carry moves up
    const uint32_t m = ((uint32_t)col[s] * BlsFp::PINV) & BlsFp::MASK;
#pragma unroll
    for (int j = 0; j < N; j++) col[s + j] += (uint64_t)m * BlsFp::P[j];
    col[s + 1] += col[s] >> BlsFp::LB;
  }
  fp x;
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < N - 1; k++) {
    c += col[k + 2];
    x.v[k] = (uint32_t)c & BlsFp::MASK;
    c >>= BlsFp::LB;
  }
  x.v[N - 1] = (uint32_t)c;
  fp_reduce_once(x, x);
  fp_to_words(out, x);
}

// One block handles BLK consecutive points. Records are packed at 96 / 192 B (in) and 104 / 200
// B (out), which lane-per-record accesses would touch at a 96-200 B stride; instead the block
// stages its whole input and output slab through LDS so that every global access is a
// contiguous, fully coalesced 16-B-per-lane sweep.
//   NC = coordinates per point (2: G1, 4: G2); the last one carries the SWFlags.
template <int NC, int BLK>
__global__ void __launch_bounds__(BLK) k_load(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n,
                                              unsigned long long* __restrict__ first_bad,
                                              uint8_t* __restrict__ status) {
  constexpr int RIN = 48 * NC, ROUT = 48 * NC + 8;
  static_assert(RIN % 16 == 0 && (BLK * ROUT) % 16 == 0 && ROUT % 8 == 0, "slab alignment");
  __shared__ uint4 slab[BLK * ROUT / 16];
  const uint64_t base = (uint64_t)blockIdx.x * BLK;
  const int cnt = (int)((n - base) < (uint64_t)BLK ? (n - base) : (uint64_t)BLK);
  const int t = threadIdx.x;

  const uint4* src = in + base * (RIN / 16);
  const int nin = cnt * (RIN / 16);
  for (int k = t; k < nin; k += BLK) slab[k] = src[k];
  __syncthreads();

  int st = 0;
  bool finf = false;
  words res[NC];
  if (t < cnt) {
    const uint4* rec = slab + t * (RIN / 16);
    words c;
    load_le(c, rec + 3 * (NC - 1));
    const uint32_t yb = c[11] >> 24;
    const bool fpos = yb & 0x80u;
    finf = yb & 0x40u;
    // ark reads the coordinates in order; the flags are parsed before the last one's range check
#pragma unroll
    for (int k = 0; k < NC - 1; k++) {
      words a;
      load_le(a, rec + 3 * k);
      if (!st && words_geq_p(a)) st = 3;
    }
    if (!st && fpos && finf) st = 6;
    c[11] &= 0x3fffffffu;
    if (!st && words_geq_p(c)) st = 3;
#pragma clang loop unroll(full)
    for (int k = 0; k < NC; k++) {
      words a;
      load_le(a, rec + 3 * k);
      if (k == NC - 1) a[11] &= 0x3fffffffu;
      words_to_ark_mont(res[k], a);
    }
  }
  __syncthreads();  // every lane has read its input record: the slab becomes the output slab
  if (t < cnt) {
    uint2* dst = (uint2*)slab + t * (ROUT / 8);
#pragma unroll
    for (int k = 0; k < NC; k++)
#pragma unroll
      for (int j = 0; j < 6; j++) dst[6 * k + j] = st ? make_uint2(0, 0) : make_uint2(res[k][2 * j], res[k][2 * j + 1]);
    dst[6 * NC] = make_uint2((!st && finf) ? 1u : 0u, 0u);
    report(base + t, st, first_bad, status);
  }
  __syncthreads();
  if (cnt == BLK) {
    uint4* dst = (uint4*)((uint8_t*)out + base * ROUT);  // BLK * ROUT is a multiple of 16
    for (int k = t; k < BLK * ROUT / 16; k += BLK) dst[k] = slab[k];
  } else {  // ragged tail block: the slab ends on an 8-B boundary
    uint2* dst = (uint2*)out + base * (ROUT / 8);
    const uint2* s2 = (const uint2*)slab;
    for (int k = t; k < cnt * (ROUT / 8); k += BLK) dst[k] = s2[k];
  }
}

hipError_t launch_load(bool g2, const void* d_in, void* d_out, uint64_t n, unsigned long long* d_first_bad,
                       uint8_t* d_status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (g2) {
    constexpr int B = 128;
    hipLaunchKernelGGL((k_load<4, B>), dim3((unsigned)((n + B - 1) / B)), dim3(B), 0, stream, (const uint4*)d_in,
                       (uint4*)d_out, n, d_first_bad, d_status);
  } else {
    constexpr int B = 256;
    hipLaunchKernelGGL((k_load<2, B>), dim3((unsigned)((n + B - 1) / B)), dim3(B), 0, stream, (const uint4*)d_in,
                       (uint4*)d_out, n, d_first_bad, d_status);
  }
  return hipGetLastError();
}

}  // namespace kzgpot
