// The hot path: one lane per point, decompress -> check -> arkworks emit. Checked streams (the
// headline) run both phases in ONE kernel (k_g1_codec in g1_kernels.hip, k_g2_codec below);
// unchecked streams run phase 1 alone, and the KZGPOT_SPLIT_PHASES A/B mode runs the two phases as
// two kernels.
//
// Replaces, per point, the reference's three CPU passes:
//   powersoftau Accumulator::deserialize → pairing into_affine_unchecked   (preprocess-kgz.rs:105)
//   Accumulator::serialize(UseCompression::No) → 1.2 GB intermediate file   (preprocess-kgz.rs:122)
//   read_g1 / read_g2 → ark deserialize_uncompressed (subgroup check)     (src/lib.rs:41-80)
//   serialize_uncompressed into the kzg_setup file                       (preprocess-kgz.rs:188-194)
// The intermediate never exists: for a finite point the ark bytes are the per-coordinate byte
// reversal of the pairing bytes (G2 also swaps c0/c1), so phase 1 emits them directly and phase 2
// checks them in place.
//
//   phase 1  k_gX_decompress : flags, x < p, Fp/Fp2 square root, sign rule → ark record
//                              (rejected points get a poison record: x's top limb = 0xffffffff)
//   phase 2  k_gX_check<Src> : ark deserialize_uncompressed on the record — x, y < p, SWFlags,
//                              subgroup — in place on phase 1's output (Src = ArkInPlace), or on a
//                              pairing-uncompressed input for the read_g1/read_g2 transcode
//                              (Src = PairingBE). Rejected records are zero-filled.
// Splitting the phases keeps each kernel's live register set to one algorithm (the square-root
// table or the scalar-multiplication state, not both); the extra traffic is one 96/192-B re-read
// per point, against ~1,500 Fp multiplies of work. For G1 the fused kernel parks x and y in LDS
// between the phases instead and measured the same time as the split pair on one box (2,264 vs
// 2,265 ms per 2^27 points, VALU-bound either way) with 144 instead of 263 B/point of HBM traffic.
//
// HBM layout: packed records, no padding — G1 in 48 B (3 x 16-B loads per lane), out 96 B
// (6 x 16-B stores); G2 in 96 B / out 192 B. All records are 16-B aligned.
//
// Status per point (first_bad = min index with a nonzero status, deterministic — the reference
// keeps an arbitrary one under a Mutex and then panics):
//   1 UnexpectedCompressionMode  2 UnexpectedInformation  3 NotInField  4 NotOnCurve
//   5 NotInSubgroup  6 UnexpectedFlags  7 Infinity (reference panics: read_g1 sees x >= p)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec.hpp"
#include "curve.hpp"
#include "records.hpp"

namespace kzgpot {

// ================================================================================ phase 1: G2
// Fp2 square root without Algorithm 9's data-dependent branches (any root works: the sign
// rule normalises it). With N = a0^2 + a1^2 (a is a square in Fp2 iff N is one in Fp):
//   gam = N^((p+1)/4); d = (a0 + gam)/2 (d = a0 if that is 0); t = d^((p-3)/4); s = t d
//   s^2 == d  ->  y = (s, a1 t / 2)      else (s^2 = -d, t s = -1)  ->  y = (-a1 t / 2, s)
// and a is accepted iff gam^2 == N. That one Fp squaring decides exactly what y^2 == a would
// (an Fp2 squaring, two subtractions and two zero tests, ~1.6 K VALU instructions more): for
// d != 0 both cases give y^2 = d - a1^2 / (4d) + a1 u, whose real part is a0 iff
// (a0 + gam)^2 - 2 a0 (a0 + gam) - a1^2 = gam^2 - N = 0; for d = a0 + gam = 0 (so gam = -a0) the
// fallback d = a0 gives y^2 = a iff a1 = 0 iff gam^2 = a0^2 = N (and a0 = 0 forces a = 0, y = 0).
// tests/test_fast_paths_math.py checks the equivalence against Algorithm 9. The halvings are
// fp_half (a shift) instead of multiplies by 1/2. Two Fp exponentiations (~920 Fp multiplies)
// where Algorithm 9 needs two Fp2 ones (~2,700). In: a reduced; out: y reduced.
KZG_DEV bool fp2_sqrt(fp2& y, const fp2& a) {
  fp nrm, t0, gam, d, s, h;
  fp_sqr(nrm, a.c0);
  fp_sqr(t0, a.c1);
  fp_add_nr(nrm, nrm, t0);
  fp_pow_pm3d4(t0, nrm);
  fp_mul(gam, t0, nrm);
  fp_sqr(t0, gam);
  const bool square = fp_eq(t0, nrm);  // gam^2 == N
  fp_add_nr(d, a.c0, gam);
  fp_norm(d, d);
  fp_half(d, d);  // (a0 + gam) / 2
  fp_select(d, fp_is_zero(d), a.c0, d);
  fp_pow_pm3d4(t0, d);  // t
  fp_mul(s, t0, d);
  fp_half(h, a.c1);
  fp_mul(h, h, t0);  // a1 t / 2
  fp_sqr(t0, s);
  const bool case1 = fp_eq(t0, d);
  fp nh;
  fp_zero(nh);
  fp_sub_red(nh, nh, h);
  fp_select(y.c0, case1, s, nh);
  fp_select(y.c1, case1, h, s);
  return square;
}

// x^3 + 4 (1 + u), reduced
KZG_DEV void g2_rhs(fp2& r, const fp2& x) {
  fp2 t;
  f_sqr(t, x);
  f_mul(r, t, x);
  fp four;
  fp_set(four, FP_FOUR);
  fp_add_red(r.c0, r.c0, four);
  fp_add_red(r.c1, r.c1, four);
}

__global__ void __launch_bounds__(kBlock) k_g2_decompress(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                          uint64_t n, uint32_t flags,
                                                          unsigned long long* __restrict__ first_bad,
                                                          uint8_t* __restrict__ status) {
  __shared__ uint32_t xpark[24][kBlock];  // x's canonical words across the square root (no HBM re-read)
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const bool checked = !(flags & KZGPOT_NO_SUBGROUP_CHECK);
  int st = 0;
  bool is_inf, greatest;
  fp2 a;
  {
    words w1, w0;  // wire order: x.c1 ‖ x.c0
    load_be(w1, in + i * 6);
    load_be(w0, in + i * 6 + 3);
    const uint32_t b0 = w1[11] >> 24;
    uint32_t rest = w0[11];
#pragma unroll
    for (int k = 0; k < 11; k++) rest |= w1[k] | w0[k];
    const bool inf_clean = ((w1[11] & 0x3fffffffu) | rest) == 0;
    w1[11] &= 0x1fffffffu;
    if (!(b0 & 0x80u)) st = 1;
    else if (b0 & 0x40u) st = inf_clean ? (checked ? 7 : 0) : 2;
    else if (words_geq_p(w0) || words_geq_p(w1)) st = 3;
    is_inf = (b0 & 0xc0u) == 0xc0u && st == 0;
    greatest = (b0 & 0x20u) != 0;
#pragma unroll
    for (int k = 0; k < 12; k++) xpark[k][threadIdx.x] = w0[k], xpark[12 + k][threadIdx.x] = w1[k];
    fp2 x;
    words_to_mont(x.c0, w0);
    words_to_mont(x.c1, w1);
    g2_rhs(a, x);
  }
  fp2 y;
  const bool on = fp2_sqrt(y, a);
  if (st == 0 && !is_inf && !on) st = 4;

  // pairing Ord for Fq2: lexicographic, c1 first
  fp2 yc, nyc;
  fp_from_mont(yc.c0, y.c0);
  fp_from_mont(yc.c1, y.c1);
  fp_neg_canon(nyc.c0, yc.c0);
  fp_neg_canon(nyc.c1, yc.c1);
  bool c1eq = true;
#pragma unroll
  for (int k = 0; k < NL; k++) c1eq = c1eq && (yc.c1.v[k] == nyc.c1.v[k]);
  const bool lt = c1eq ? fp_lt_canon(yc.c0, nyc.c0) : fp_lt_canon(yc.c1, nyc.c1);
  const bool keep = lt ^ greatest;

  uint4* dst = out + i * 12;
  if (st == 0 && !is_inf) {
    words w1, w0;
    uint32_t lane = threadIdx.x;
    asm volatile("" : "+v"(lane));
#pragma unroll
    for (int k = 0; k < 12; k++) w0[k] = xpark[k][lane], w1[k] = xpark[12 + k][lane];
    fp_select(yc.c0, keep, yc.c0, nyc.c0);
    fp_select(yc.c1, keep, yc.c1, nyc.c1);
    store_words(dst, w0);
    store_words(dst + 3, w1);
    store_canon(dst + 6, yc.c0);
    store_canon(dst + 9, yc.c1);
  } else {
    words z, zx, zy0, zy1;
    zero_words(z);
    zero_words(zx);
    zero_words(zy0);
    zero_words(zy1);
    if (is_inf) zy0[0] = 1, zy1[11] = 0x40000000u;  // ark zero() = ((0,0), (1,0), inf)
    if (st && checked) zx[11] = kPoison;
    store_words(dst, zx);
    store_words(dst + 3, z);
    store_words(dst + 6, zy0);
    store_words(dst + 9, zy1);
  }
  report(i, st, first_bad, status);
}

// ================================================================================ fused G2 codec
// Both phases of a checked G2 point in one lane and one launch, as k_g1_codec: x's Montgomery
// form is parked in LDS before the square root (its canonical words wait in y's slots, which are
// free until the emit), the ark record goes out in one go after the sign rule, and y's Montgomery
// form replaces the words. The ladder reads the base point from LDS. The split path's check
// re-reads the 192-B record, converts four coordinates and tests the curve equation; here the
// point is on the curve by construction (fp2_sqrt accepts only when y^2 = x^3 + 4 (1 + u)) and only y is
// converted. 56 KB of LDS per block.
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_g2_codec(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n, uint32_t flags,
           unsigned long long* __restrict__ first_bad, uint8_t* __restrict__ status) {
  __shared__ uint32_t base[4 * NL][kBlock];  // x.c0, x.c1, y.c0, y.c1 (Montgomery), limb-major
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  int st = 0;
  bool greatest;
  uint4* dst = out + i * 12;
  fp2 a;
  {
    words w1, w0;  // wire order: x.c1 ‖ x.c0
    load_be(w1, in + i * 6);
    load_be(w0, in + i * 6 + 3);
    const uint32_t b0 = w1[11] >> 24;
    uint32_t rest = w0[11];
#pragma unroll
    for (int k = 0; k < 11; k++) rest |= w1[k] | w0[k];
    const bool inf_clean = ((w1[11] & 0x3fffffffu) | rest) == 0;
    w1[11] &= 0x1fffffffu;
    if (!(b0 & 0x80u)) st = 1;
    else if (b0 & 0x40u) st = inf_clean ? 7 : 2;  // checked stream: infinity is rejected
    else if (words_geq_p(w0) || words_geq_p(w1)) st = 3;
    greatest = (b0 & 0x20u) != 0;
#pragma unroll
    for (int k = 0; k < 12; k++) base[2 * NL + k][threadIdx.x] = w0[k], base[2 * NL + 12 + k][threadIdx.x] = w1[k];
    fp2 x;
    words_to_mont(x.c0, w0);
    words_to_mont(x.c1, w1);
#pragma unroll
    for (int k = 0; k < NL; k++) base[k][threadIdx.x] = x.c0.v[k], base[NL + k][threadIdx.x] = x.c1.v[k];
    g2_rhs(a, x);
  }
  {
    fp2 y;
    const bool on = fp2_sqrt(y, a);
    if (st == 0 && !on) st = 4;
    fp2 yc, nyc;
    fp_from_mont(yc.c0, y.c0);
    fp_from_mont(yc.c1, y.c1);
    fp_neg_canon(nyc.c0, yc.c0);
    fp_neg_canon(nyc.c1, yc.c1);
    bool c1eq = true;
#pragma unroll
    for (int k = 0; k < NL; k++) c1eq = c1eq && (yc.c1.v[k] == nyc.c1.v[k]);
    const bool keep = (c1eq ? fp_lt_canon(yc.c0, nyc.c0) : fp_lt_canon(yc.c1, nyc.c1)) ^ greatest;
    if (st == 0) {
      words w0, w1;
      uint32_t lane = threadIdx.x;
      asm volatile("" : "+v"(lane));
#pragma unroll
      for (int k = 0; k < 12; k++) w0[k] = base[2 * NL + k][lane], w1[k] = base[2 * NL + 12 + k][lane];
      fp_select(yc.c0, keep, yc.c0, nyc.c0);
      fp_select(yc.c1, keep, yc.c1, nyc.c1);
      store_words(dst, w0);
      store_words(dst + 3, w1);
      store_canon(dst + 6, yc.c0);
      store_canon(dst + 9, yc.c1);
      // the chosen root in Montgomery form for the ladder: y's representative made canonical, or
      // its negation p - y (0 -> 0), instead of converting the canonical bytes back (two multiplies)
      fp m;
      fp_reduce_once(y.c0, y.c0);
      fp_neg_canon(m, y.c0);
      fp_select(y.c0, keep, y.c0, m);
      fp_reduce_once(y.c1, y.c1);
      fp_neg_canon(m, y.c1);
      fp_select(y.c1, keep, y.c1, m);
#pragma unroll
      for (int k = 0; k < NL; k++) base[2 * NL + k][threadIdx.x] = y.c0.v[k], base[3 * NL + k][threadIdx.x] = y.c1.v[k];
    }
  }
  if (st == 0) {
    auto load = [&](fp2& bx, fp2& by) {
      uint32_t lane = threadIdx.x;
      asm volatile("" : "+v"(lane));  // opaque index: re-read at every use, never hoisted
#pragma unroll
      for (int k = 0; k < NL; k++) {
        bx.c0.v[k] = base[k][lane];
        bx.c1.v[k] = base[NL + k][lane];
        by.c0.v[k] = base[2 * NL + k][lane];
        by.c1.v[k] = base[3 * NL + k][lane];
      }
    };
    const bool ok = (flags & KZGPOT_SUBGROUP_REF) ? in_subgroup_ref<fp2>(load) : in_subgroup_fast_g2(load);
    if (!ok) st = 5;
  }
  if (st) store_zero(dst, 12);
  report(i, st, first_bad, status);
}

// ================================================================================ phase 2
// ark-ec 0.2 deserialize_uncompressed on one record, then serialize_uncompressed.
//   Src::ArkInPlace : the record is phase 1's output (ark LE, x ‖ y)           — decompress path
//   Src::PairingBE  : pairing-uncompressed input; read_g1 (src/lib.rs:41-54) / read_g2
//                     (src/lib.rs:56-80) byte order is applied on load        — transcode path
//   Src::PairingBEInPlace : the same, reading and rewriting the records of `out` (load_phase1's
//                     first stage; no restrict-qualified pointer aliases another)
// The reference checks no curve equation: points on the curve take the endomorphism test, the
// rest the exact ark double-and-add by r (divergent, but only for inputs that are not points).

template <Src S>
struct G2Rec {
  // x.c0, x.c1, y.c0, y.c1 as words
  static KZG_DEV void load_xy(words& x0, words& x1, words& y0, words& y1, const uint4* rec) {
    if constexpr (S == Src::ArkInPlace) {  // x.c0, x.c1, y.c0, y.c1 (LE)
      load_le(x0, rec);
      load_le(x1, rec + 3);
      load_le(y0, rec + 6);
      load_le(y1, rec + 9);
    } else {  // wire: x.c1, x.c0, y.c1, y.c0 (BE)
      load_be(x1, rec);
      load_be(x0, rec + 3);
      load_be(y1, rec + 6);
      load_be(y0, rec + 9);
    }
  }
};

template <Src S>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_g2_check(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n, uint32_t flags,
           unsigned long long* __restrict__ first_bad, uint8_t* __restrict__ status) {
  __shared__ uint32_t base[4 * NL][kBlock];  // Montgomery base point, limb-major (see k_g1_check, g1_kernels.hip)
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint4* rec = (src_in_place(S) ? (const uint4*)out : in) + i * 12;
  uint4* dst = out + i * 12;
  int st = 0;
  bool finf;
  {
    // one read of the record; a transcode record is emitted before the test (see k_g1_check, g1_kernels.hip)
    words x0, x1, y0, y1;
    G2Rec<S>::load_xy(x0, x1, y0, y1, rec);
    if (S == Src::ArkInPlace && x0[11] == kPoison) {
      store_zero(dst, 12);
      return;
    }
    const uint32_t yb = y1[11] >> 24;
    const bool fpos = yb & 0x80u;
    finf = yb & 0x40u;
    y1[11] &= 0x3fffffffu;
    if (words_geq_p(x0) || words_geq_p(x1)) st = 3;
    else if (words_geq_p(y0)) st = 3;
    else if (fpos && finf) st = 6;
    else if (words_geq_p(y1)) st = 3;
    if (S != Src::ArkInPlace && st == 0) {
      store_words(dst, x0);
      store_words(dst + 3, x1);
      store_words(dst + 6, y0);
      words e;
#pragma unroll
      for (int k = 0; k < 12; k++) e[k] = y1[k];
      if (finf) e[11] |= 0x40000000u;
      store_words(dst + 9, e);
    }
    if (st == 0 && !finf) {
      fp t;
      words_to_mont(t, x0);
#pragma unroll
      for (int k = 0; k < NL; k++) base[k][threadIdx.x] = t.v[k];
      words_to_mont(t, x1);
#pragma unroll
      for (int k = 0; k < NL; k++) base[NL + k][threadIdx.x] = t.v[k];
      words_to_mont(t, y0);
#pragma unroll
      for (int k = 0; k < NL; k++) base[2 * NL + k][threadIdx.x] = t.v[k];
      words_to_mont(t, y1);
#pragma unroll
      for (int k = 0; k < NL; k++) base[3 * NL + k][threadIdx.x] = t.v[k];
    }
  }

  if (st == 0 && !finf) {
    auto load = [&](fp2& bx, fp2& by) {
      uint32_t lane = threadIdx.x;
      asm volatile("" : "+v"(lane));  // opaque index: re-read at every use, never hoisted
#pragma unroll
      for (int k = 0; k < NL; k++) {
        bx.c0.v[k] = base[k][lane];
        bx.c1.v[k] = base[NL + k][lane];
        by.c0.v[k] = base[2 * NL + k][lane];
        by.c1.v[k] = base[3 * NL + k][lane];
      }
    };
    bool on_curve;
    {
      fp2 xm, ym, l, r;
      load(xm, ym);
      f_sqr(l, ym);
      g2_rhs(r, xm);
      fp_sub_red(l.c0, l.c0, r.c0);
      fp_sub_red(l.c1, l.c1, r.c1);
      on_curve = f_is_zero(l);
    }
    bool ok;
    if ((flags & KZGPOT_SUBGROUP_REF) || !on_curve)
      ok = in_subgroup_ref<fp2>(load);
    else
      ok = in_subgroup_fast_g2(load);
    if (!ok) st = 5;
  }
  if (st) store_zero(dst, 12);
  report(i, st, first_bad, status);
}

// ================================================================================ launchers
static inline unsigned grid_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

hipError_t launch_codec(CodecOp op, const void* d_in, void* d_out, uint64_t n, uint32_t flags,
                        unsigned long long* d_first_bad, uint8_t* d_status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const dim3 grid(grid_for(n)), block(kBlock);
  const uint4* in = (const uint4*)d_in;
  uint4* out = (uint4*)d_out;
  const bool checked = !(flags & KZGPOT_NO_SUBGROUP_CHECK);
  switch (op) {
    case CodecOp::G1Decompress:
    case CodecOp::G1Transcode:
      return launch_g1(op, in, out, n, flags, d_first_bad, d_status, stream);
    case CodecOp::G2Decompress:
      if (checked && !(flags & KZGPOT_SPLIT_PHASES)) {
        hipLaunchKernelGGL(k_g2_codec, grid, block, 0, stream, in, out, n, flags, d_first_bad, d_status);
        break;
      }
      hipLaunchKernelGGL(k_g2_decompress, grid, block, 0, stream, in, out, n, flags, d_first_bad, d_status);
      if (checked)
        hipLaunchKernelGGL(k_g2_check<Src::ArkInPlace>, grid, block, 0, stream, in, out, n, flags, d_first_bad,
                           d_status);
      break;
    case CodecOp::G2Transcode:
      hipLaunchKernelGGL(k_g2_check<Src::PairingBE>, grid, block, 0, stream, in, out, n, flags, d_first_bad,
                         d_status);
      break;
    case CodecOp::G1Phase1: {  // read_g1 in place on the (caller-owned staging) input, then GroupAffine
      const hipError_t e = launch_g1(op, nullptr, (uint4*)d_in, n, flags, d_first_bad, d_status, stream);
      if (e != hipSuccess) return e;
      return launch_load(false, d_in, d_out, n, d_first_bad, nullptr, stream);
    }
    case CodecOp::G2Phase1:
      hipLaunchKernelGGL(k_g2_check<Src::PairingBEInPlace>, grid, block, 0, stream, nullptr, (uint4*)d_in, n, flags,
                         d_first_bad, d_status);
      return launch_load(true, d_in, d_out, n, d_first_bad, nullptr, stream);
    case CodecOp::G1Load:
    case CodecOp::G2Load:
      return launch_load(op == CodecOp::G2Load, d_in, d_out, n, d_first_bad, d_status, stream);
    case CodecOp::Bn254G1Decompress:
      return launch_bn254(d_in, d_out, n, d_first_bad, d_status, stream);
  }
  return hipGetLastError();
}

}  // namespace kzgpot
