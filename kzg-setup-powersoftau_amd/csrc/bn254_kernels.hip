// BN254 G1 point codec (config 5 / SURVEY §8f row 4 — no reference counterpart; the format is
// the arkworks one the reference already uses for BLS12-381, instantiated for ark-bn254 0.2):
//   in : ark compressed G1, 32 B — x little-endian, SWFlags in the top 2 bits of byte 31
//        (bit 7 PositiveY = "y > -y", bit 6 Infinity)
//   out: ark uncompressed G1, 64 B — x LE ‖ y LE (no flags for a finite point; the point at
//        infinity is ark zero() = (0, 1) with bit 6 of byte 63 set)
// i.e. ark-ec 0.2 `GroupAffine::deserialize` then `serialize_uncompressed`:
//   flags both set → UnexpectedFlags; x >= p → InvalidData (NotInField); Infinity → zero();
//   else get_point_from_x(x, PositiveY): y = sqrt(x^3 + 3) (none → NotOnCurve), keep y if
//   (y < -y) XOR PositiveY else -y; subgroup check: BN254 G1 has cofactor 1, so every curve
//   point passes (ark's mul_bits(r) test is identically true there and is not run).
// One lane per point; 32 B in + 64 B out against one (p-3)/4 exponentiation over a 9 x 29-bit-limb
// field (81 products per multiply instead of 100 with 10 x 28-bit limbs).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec.hpp"
#include "fp381.hpp"
#include "records.hpp"

namespace kzgpot {

using bnwords = uint32_t[8];

KZG_DEV void load8(bnwords& w, const uint4* src) {
  const uint4 a = src[0], b = src[1];
  w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w;
  w[4] = b.x, w[5] = b.y, w[6] = b.z, w[7] = b.w;
}
KZG_DEV void store8(uint4* dst, const bnwords& w) {
  dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
  dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__global__ void __launch_bounds__(kBlock) k_bn254_g1_decompress(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                                uint64_t n, unsigned long long* __restrict__ first_bad,
                                                                uint8_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  int st = 0;
  bool inf, positive;
  fpbn a;
  {
    bnwords w;
    load8(w, in + i * 2);
    const uint32_t top = w[7] >> 24;
    positive = top & 0x80u;
    inf = top & 0x40u;
    w[7] &= 0x3fffffffu;
    if (positive && inf) st = 6;
    else if (words_geq_p_t<Bn254Fp>(w)) st = 3;
    fpbn x, t;
    fp_from_words(x, w);
    fp_to_mont(t, x);  // x < 2^254 even when rejected: bounds hold (test_field_bounds.py)
    fp_sqr(a, t);
    fp_mul(a, a, t);
    fp_set(x, BN_THREE);
    fp_add(a, a, x);  // x^3 + 3
  }
  fpbn y, t;
  fp_pow_pm3d4(t, a);
  fp_mul(y, t, a);
  fp_sqr(t, y);
  if (st == 0 && !inf && !fp_eq(t, a)) st = 4;

  fpbn yc, nyc;
  fp_from_mont(yc, y);
  fp_neg_canon(nyc, yc);
  const bool keep = fp_lt_canon(yc, nyc) ^ positive;

  uint4* dst = out + i * 4;
  bnwords w;
  if (st == 0 && !inf) {
    load8(w, opaque(in) + i * 2);
    w[7] &= 0x3fffffffu;
    store8(dst, w);
    fp_select(yc, keep, yc, nyc);
    fp_to_words(w, yc);
    store8(dst + 2, w);
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = 0;
    store8(dst, w);
    if (st == 0) w[0] = 1, w[7] = 0x40000000u;  // ark zero() = (0, 1, infinity)
    store8(dst + 2, w);
  }
  report(i, st, first_bad, status);
}

hipError_t launch_bn254(const void* d_in, void* d_out, uint64_t n, unsigned long long* d_first_bad, uint8_t* d_status,
                        hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bn254_g1_decompress, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                     (const uint4*)d_in, (uint4*)d_out, n, d_first_bad, d_status);
  return hipGetLastError();
}

}  // namespace kzgpot
