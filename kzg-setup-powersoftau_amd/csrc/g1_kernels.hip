// The G1 half of the hot path (the headline: 2^27 of the 2^27 + 2^16 points), in its own translation
// unit so that it can be compiled with its own scheduler (Makefile: -amdgpu-sched-strategy=
// iterative-ilp, -0.7 % time per G1 point on the same box; the G2 kernels measured +0.9 % with it,
// so codec_kernels.hip keeps the default). Kernels, phases, layout and status codes are described
// at the top of codec_kernels.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codec.hpp"
#include "curve.hpp"
#include "records.hpp"

namespace kzgpot {

// ================================================================================ phase 1: G1
__global__ void __launch_bounds__(kBlock) k_g1_decompress(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                          uint64_t n, uint32_t flags,
                                                          unsigned long long* __restrict__ first_bad,
                                                          uint8_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const bool checked = !(flags & KZGPOT_NO_SUBGROUP_CHECK);
  int st = 0;
  bool is_inf, greatest;
  fp a;
  {
    words w;
    load_be(w, in + i * 3);
    const uint32_t b0 = w[11] >> 24;  // first byte on the wire
    uint32_t rest = 0;
#pragma unroll
    for (int k = 0; k < 11; k++) rest |= w[k];
    const bool inf_clean = ((w[11] & 0x3fffffffu) | rest) == 0;  // copy[0] &= 0x3f; all zero?
    w[11] &= 0x1fffffffu;
    if (!(b0 & 0x80u)) st = 1;
    else if (b0 & 0x40u) st = inf_clean ? (checked ? 7 : 0) : 2;
    else if (words_geq_p(w)) st = 3;
    is_inf = (b0 & 0xc0u) == 0xc0u && st == 0;
    greatest = (b0 & 0x20u) != 0;
    fp t, u;
    words_to_mont(t, w);  // x < 2^381 even when rejected: bounds hold (test_field_bounds.py)
    fp_sqr(a, t);
    fp_mul(a, a, t);
    fp_set(u, FP_FOUR);
    fp_add(a, a, u);      // x^3 + 4
  }
  // y = (x^3 + 4)^((p+1)/4); every lane runs the same chain (wave-uniform)
  fp y, t;
  fp_pow_pm3d4(t, a);
  fp_mul(y, t, a);
  fp_sqr(t, y);
  if (st == 0 && !is_inf && !fp_eq(t, a)) st = 4;

  // sign rule (pairing get_point_from_x): keep y if (y < -y) XOR greatest, canonical order
  fp yc, nyc;
  fp_from_mont(yc, y);
  fp_neg_canon(nyc, yc);
  const bool keep = fp_lt_canon(yc, nyc) ^ greatest;

  uint4* dst = out + i * 6;
  if (st == 0 && !is_inf) {
    words w;  // re-read x rather than keep it live through the exponentiation
    load_be(w, opaque(in) + i * 3);
    w[11] &= 0x1fffffffu;
    fp_select(yc, keep, yc, nyc);
    store_words(dst, w);
    store_canon(dst + 3, yc);
  } else {
    words zx, zy;
    zero_words(zx);
    zero_words(zy);
    if (is_inf) zy[0] = 1, zy[11] = 0x40000000u;  // ark GroupAffine::zero() = (0, 1, inf)
    if (st && checked) zx[11] = kPoison;          // phase 2 zero-fills and skips it
    store_words(dst, zx);
    store_words(dst + 3, zy);
  }
  report(i, st, first_bad, status);
}

// ================================================================================ fused G1 codec
// Both phases of a checked G1 point in one lane and one launch (the default for checked
// streams): x's canonical words and its Montgomery form are parked in LDS before the square root,
// the ark record (x, y) goes out after the sign rule and y's Montgomery form is parked next to x —
// so nothing but the ladder state is live across the subgroup test,
// and no record is read back from HBM (48 B in + 96 B out per point, against 48 + 96 + 96 + the
// x re-read of the split kernels). A rejected point's record is zero-filled (the split path's
// phase 2 does the same to its poison record). 70 KB of LDS per block (base point + the second
// ladder's base, as k_g1_check) holds the kernel at 2 waves per SIMD.
__global__ void __launch_bounds__(kBlock) k_g1_codec(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                     uint64_t n, uint32_t flags,
                                                     unsigned long long* __restrict__ first_bad,
                                                     uint8_t* __restrict__ status) {
  __shared__ uint32_t base[2 * NL][kBlock];
  __shared__ uint32_t qpark[3 * NL][kBlock];
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  int st = 0;
  bool greatest;
  uint4* dst = out + i * 6;
  fp a;
  {
    words w;
    load_be(w, in + i * 3);
    const uint32_t b0 = w[11] >> 24;
    uint32_t rest = 0;
#pragma unroll
    for (int k = 0; k < 11; k++) rest |= w[k];
    const bool inf_clean = ((w[11] & 0x3fffffffu) | rest) == 0;
    w[11] &= 0x1fffffffu;
    if (!(b0 & 0x80u)) st = 1;
    else if (b0 & 0x40u) st = inf_clean ? 7 : 2;  // checked stream: infinity is rejected
    else if (words_geq_p(w)) st = 3;
    greatest = (b0 & 0x20u) != 0;
#pragma unroll
    for (int k = 0; k < 12; k++) qpark[k][threadIdx.x] = w[k];  // ark x = the canonical x (qpark is free until the ladder)
    fp t, u;
    words_to_mont(t, w);
#pragma unroll
    for (int k = 0; k < NL; k++) base[k][threadIdx.x] = t.v[k];
    fp_sqr(a, t);
    fp_mul(a, a, t);
    fp_set(u, FP_FOUR);
    fp_add(a, a, u);
  }
  {
    fp y, t;
    fp_pow_pm3d4(t, a);
    fp_mul(y, t, a);
    fp_sqr(t, y);
    if (st == 0 && !fp_eq(t, a)) st = 4;
    fp yc, nyc;
    fp_from_mont(yc, y);
    fp_neg_canon(nyc, yc);
    const bool keep = fp_lt_canon(yc, nyc) ^ greatest;
    fp_select(yc, keep, yc, nyc);
    if (st == 0) {
      words w;  // the whole 96-B record in one go: a 48-B half written long before the other costs
      uint32_t lane = threadIdx.x;  // a partial 64-B write per half (PMC: 155 instead of 96 B/point)
      asm volatile("" : "+v"(lane));
#pragma unroll
      for (int k = 0; k < 12; k++) w[k] = qpark[k][lane];
      store_words(dst, w);
      store_canon(dst + 3, yc);
      // the chosen root in Montgomery form: y's representative made canonical, or p - y (0 -> 0),
      // instead of converting the canonical bytes back (a multiply)
      fp_reduce_once(y, y);
      fp_neg_canon(t, y);
      fp_select(y, keep, y, t);
#pragma unroll
      for (int k = 0; k < NL; k++) base[NL + k][threadIdx.x] = y.v[k];
    }
  }
  if (st == 0) {
    auto load = [&](fp& bx, fp& by) {
      uint32_t lane = threadIdx.x;
      asm volatile("" : "+v"(lane));  // opaque index: re-read at every use, never hoisted
#pragma unroll
      for (int k = 0; k < NL; k++) bx.v[k] = base[k][lane], by.v[k] = base[NL + k][lane];
    };
    bool ok;
    if (flags & KZGPOT_SUBGROUP_REF) {
      ok = in_subgroup_ref<fp>(load);
    } else {
      auto park = [&](const jac<fp>& q) {
#pragma unroll
        for (int k = 0; k < NL; k++) {
          qpark[k][threadIdx.x] = q.x.v[k];
          qpark[NL + k][threadIdx.x] = q.y.v[k];
          qpark[2 * NL + k][threadIdx.x] = q.z.v[k];
        }
      };
      auto load_row = [&](int src, fp& bx, fp& by) {  // src 0: P (base), 1: Q1 (qpark); wave-uniform
        uint32_t lane = threadIdx.x;
        asm volatile("" : "+v"(lane));
        const uint32_t* b = src ? &qpark[0][0] : &base[0][0];
#pragma unroll
        for (int k = 0; k < NL; k++) bx.v[k] = b[k * kBlock + lane], by.v[k] = b[(NL + k) * kBlock + lane];
      };
      auto load_qz = [&](fp& qz) {
        uint32_t lane = threadIdx.x;
        asm volatile("" : "+v"(lane));
#pragma unroll
        for (int k = 0; k < NL; k++) qz.v[k] = qpark[2 * NL + k][lane];
      };
      ok = in_subgroup_fast_g1(load_row, park, load_qz);
    }
    if (!ok) st = 5;
  }
  if (st) store_zero(dst, 6);
  report(i, st, first_bad, status);
}

template <Src S>
struct G1Rec {
  static KZG_DEV void load_xy(words& x, words& y, const uint4* rec) {
    if constexpr (S == Src::ArkInPlace) {
      load_le(x, rec);
      load_le(y, rec + 3);
    } else {
      load_be(x, rec);
      load_be(y, rec + 3);
    }
  }
};

template <Src S>
__global__ void __launch_bounds__(kBlock) k_g1_check(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                     uint64_t n, uint32_t flags,
                                                     unsigned long long* __restrict__ first_bad,
                                                     uint8_t* __restrict__ status) {
  // The base point in Montgomery form is parked in LDS (limb-major, so the 64 lanes of a wave hit
  // 64 consecutive dwords): each of the ~8 reloads in the ladders is 28 LDS reads instead of two
  // Montgomery conversions, and the point costs no VGPRs between reloads. The fast test's second
  // ladder base Q1 = [|u|]P = (X : Y : Z) is parked beside it (qpark). 70 KB per 256-lane block:
  // 2 blocks per CU, the occupancy the VGPR count allows anyway.
  __shared__ uint32_t base[2 * NL][kBlock];
  __shared__ uint32_t qpark[3 * NL][kBlock];
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint4* rec = (src_in_place(S) ? (const uint4*)out : in) + i * 6;
  uint4* dst = out + i * 6;
  int st = 0;
  bool finf;
  {
    // The record is read ONCE: a transcode record that passes the flag and field checks is
    // emitted right away (as k_g1_codec emits before its subgroup test) and zero-filled if the
    // test rejects it, so nothing is re-read from HBM after the ladders (192 B/point moved).
    words x, y;
    G1Rec<S>::load_xy(x, y, rec);
    if (S == Src::ArkInPlace && x[11] == kPoison) {  // phase 1 already rejected (and reported) it
      store_zero(dst, 6);
      return;
    }
    const uint32_t yb = y[11] >> 24;  // ark SWFlags: top byte of y
    const bool fpos = yb & 0x80u;
    finf = yb & 0x40u;
    y[11] &= 0x3fffffffu;
    if (words_geq_p(x)) st = 3;
    else if (fpos && finf) st = 6;
    else if (words_geq_p(y)) st = 3;
    if (S != Src::ArkInPlace && st == 0) {
      words e;
#pragma unroll
      for (int k = 0; k < 12; k++) e[k] = y[k];
      if (finf) e[11] |= 0x40000000u;  // GroupAffine::new(x, y, true) keeps x, y
      store_words(dst, x);
      store_words(dst + 3, e);
    }
    if (st == 0 && !finf) {
      fp bx, by;
      words_to_mont(bx, x);
      words_to_mont(by, y);
#pragma unroll
      for (int k = 0; k < NL; k++) base[k][threadIdx.x] = bx.v[k], base[NL + k][threadIdx.x] = by.v[k];
    }
  }

  if (st == 0 && !finf) {
    auto load = [&](fp& bx, fp& by) {
      uint32_t lane = threadIdx.x;
      asm volatile("" : "+v"(lane));  // opaque index: re-read at every use, never hoisted
#pragma unroll
      for (int k = 0; k < NL; k++) bx.v[k] = base[k][lane], by.v[k] = base[NL + k][lane];
    };
    // Phase 1 emits only points with y^2 = x^3 + 4 (it rejects non-residues), so an in-place
    // record is on the curve; a transcode input may not be (the reference never checks).
    bool on_curve = true;
    if (S != Src::ArkInPlace) {
      fp xm, ym, l, r;
      load(xm, ym);
      fp_sqr(l, ym);
      fp_sqr(r, xm);
      fp_mul(r, r, xm);
      fp_set(xm, FP_FOUR);
      fp_add(r, r, xm);
      on_curve = fp_eq(l, r);
    }
    bool ok;
    if ((flags & KZGPOT_SUBGROUP_REF) || !on_curve) {
      ok = in_subgroup_ref<fp>(load);
    } else {
      auto park = [&](const jac<fp>& q) {
#pragma unroll
        for (int k = 0; k < NL; k++) {
          qpark[k][threadIdx.x] = q.x.v[k];
          qpark[NL + k][threadIdx.x] = q.y.v[k];
          qpark[2 * NL + k][threadIdx.x] = q.z.v[k];
        }
      };
      auto load_row = [&](int src, fp& bx, fp& by) {  // src 0: P (base), 1: Q1 (qpark); wave-uniform
        uint32_t lane = threadIdx.x;
        asm volatile("" : "+v"(lane));
        const uint32_t* b = src ? &qpark[0][0] : &base[0][0];
#pragma unroll
        for (int k = 0; k < NL; k++) bx.v[k] = b[k * kBlock + lane], by.v[k] = b[(NL + k) * kBlock + lane];
      };
      auto load_qz = [&](fp& qz) {
        uint32_t lane = threadIdx.x;
        asm volatile("" : "+v"(lane));
#pragma unroll
        for (int k = 0; k < NL; k++) qz.v[k] = qpark[2 * NL + k][lane];
      };
      ok = in_subgroup_fast_g1(load_row, park, load_qz);
    }
    if (!ok) st = 5;
  }
  if (st) store_zero(dst, 6);
  report(i, st, first_bad, status);
}

// ================================================================================ launcher
hipError_t launch_g1(CodecOp op, const uint4* in, uint4* out, uint64_t n, uint32_t flags,
                     unsigned long long* d_first_bad, uint8_t* d_status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock)), block(kBlock);
  const bool checked = !(flags & KZGPOT_NO_SUBGROUP_CHECK);
  switch (op) {
    case CodecOp::G1Decompress:
      if (checked && !(flags & KZGPOT_SPLIT_PHASES)) {
        hipLaunchKernelGGL(k_g1_codec, grid, block, 0, stream, in, out, n, flags, d_first_bad, d_status);
        break;
      }
      hipLaunchKernelGGL(k_g1_decompress, grid, block, 0, stream, in, out, n, flags, d_first_bad, d_status);
      if (checked)
        hipLaunchKernelGGL(k_g1_check<Src::ArkInPlace>, grid, block, 0, stream, in, out, n, flags, d_first_bad,
                           d_status);
      break;
    case CodecOp::G1Transcode:
      hipLaunchKernelGGL(k_g1_check<Src::PairingBE>, grid, block, 0, stream, in, out, n, flags, d_first_bad,
                         d_status);
      break;
    case CodecOp::G1Phase1:
      hipLaunchKernelGGL(k_g1_check<Src::PairingBEInPlace>, grid, block, 0, stream, nullptr, out, n, flags,
                         d_first_bad, d_status);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kzgpot
