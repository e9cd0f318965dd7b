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
// HBM-bound: 96 B in + 104 B out per G1 point against 2 Fp multiplies. The product kernel is
// k_load_direct (below): each lane reads one coordinate straight from HBM, and the output is staged
// through LDS so that its stores are fully coalesced.
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
// The final conditional subtraction is needed only when the result's top limb reaches p's
// (the value is < 1.000001 p, so a top limb below p's means a value below p; a uniform value hits
// it with probability ~1e-5): FILTER runs it in a wave-uniform branch taken only when some lane of
// the wave needs it, 56 instructions per lane saved otherwise. FILTER = false: the r06n form (the
// microbenchmark's A sides).
template <bool FILTER = true>
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
  if (!FILTER || __ballot(x.v[N - 1] >= BlsFp::P[N - 1])) fp_reduce_once(x, x);
  fp_to_words(out, x);
}


// k_load: the product loader of rounds 2-5, kept for tools/microbench/loader_ceiling.hip.
// One block handles PTS consecutive points. Records are packed at 96 / 192 B (in) and 104 / 200
// B (out), which lane-per-record accesses would touch at a 96-200 B stride; instead the block
// stages its whole input and output slab through LDS so that every global access is a
// contiguous, fully coalesced 16-B-per-lane sweep.
// A point is a lane pair: G1 one coordinate per lane (x; y with the flags), G2 two (x.c0 x.c1;
// y.c0 y.c1 with the flags). G2 at one lane per point held 4 conversions per lane and only 3
// waves per SIMD (LDS-bound: 200 B of slab per point): 3.8-4.0 TB/s, 5.3-5.4 as lane pairs. G1 as
// lane pairs of 128-point blocks: 5.56 against 5.45-5.50 TB/s at one lane per point (256- or
// 128-point blocks), same box (profiles/r03_loader_ceiling.txt) — shorter per-block compute
// overlaps the other blocks' sweeps better.
// The global sweeps are nontemporal (streaming: neither slab is read again by this kernel, and
// the output is not re-read by the next): 5.54 -> 5.96 TB/s for the bare staging pattern, 5.34 ->
// 5.51 TB/s for k_load<G1> (tools/microbench/loader_ceiling.hip, profiles/r03_loader_ceiling.txt).
//   NC = coordinates per point (2: G1, 4: G2); the last one carries the SWFlags.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // the nontemporal builtins want a vector type
KZG_DEV uint4 ld_stream(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
KZG_DEV void st_stream(uint4* p, const uint4& v) { __builtin_nontemporal_store((u32x4){v.x, v.y, v.z, v.w}, (u32x4*)p); }

template <int NC, int PTS, bool NT = true, int CPL = 2>
__global__ void __launch_bounds__(PTS * NC / CPL) k_load(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                         uint64_t n, unsigned long long* __restrict__ first_bad,
                                                         uint8_t* __restrict__ status) {
  constexpr int LPP = NC / CPL, BLK = PTS * LPP;  // lanes per point; lanes per block
  constexpr int RIN = 48 * NC, ROUT = 48 * NC + 8;
  static_assert(LPP == 1 || LPP == 2, "a point is one lane or a lane pair");
  static_assert(RIN % 16 == 0 && (PTS * ROUT) % 16 == 0 && ROUT % 8 == 0, "slab alignment");
  __shared__ uint4 slab[PTS * ROUT / 16];
  const uint64_t base = (uint64_t)blockIdx.x * PTS;
  const int cnt = (int)((n - base) < (uint64_t)PTS ? (n - base) : (uint64_t)PTS);
  const int t = threadIdx.x;
  const int pt = t / LPP, h = t % LPP;  // this lane: point pt, coordinates CPL h .. CPL h + CPL - 1

  const uint4* src = in + base * (RIN / 16);
  const int nin = cnt * (RIN / 16);
  for (int k = t; k < nin; k += BLK) slab[k] = NT ? ld_stream(src + k) : src[k];
  __syncthreads();

  int st = 0;
  bool finf = false;
  words res[CPL];
  if (pt < cnt) {
    // ark reads the coordinates in order, and parses the flags before the last one's range
    // check: the lane holding the last coordinate checks its others, the flags, then the last;
    // the first lane of a pair takes precedence (its coordinates come first).
    const uint4* rec = slab + pt * (RIN / 16) + 3 * CPL * h;
    const bool last = h == LPP - 1;
    words c[CPL];
#pragma unroll
    for (int k = 0; k < CPL; k++) load_le(c[k], rec + 3 * k);
    const uint32_t yb = c[CPL - 1][11] >> 24;
    const bool fpos = yb & 0x80u;
    finf = last && (yb & 0x40u);
    if (last) c[CPL - 1][11] &= 0x3fffffffu;
    if (CPL == 2 && words_geq_p(c[0])) st = 3;
    else if (last && fpos && finf) st = 6;
    else if (words_geq_p(c[CPL - 1])) st = 3;
#pragma unroll
    for (int k = 0; k < CPL; k++) words_to_ark_mont(res[k], c[k]);
  }
  if (LPP == 2) {  // the point's status: the first lane's, else the second's (both lanes agree)
    const int other = __shfl_xor(st, 1);
    st = h == 0 ? (st ? st : other) : (other ? other : st);
  }
  __syncthreads();  // every lane has read its input record: the slab becomes the output slab
  if (pt < cnt) {
    uint2* dst = (uint2*)slab + pt * (ROUT / 8) + 6 * CPL * h;
#pragma unroll
    for (int k = 0; k < CPL; k++)
#pragma unroll
      for (int j = 0; j < 6; j++) dst[6 * k + j] = st ? make_uint2(0, 0) : make_uint2(res[k][2 * j], res[k][2 * j + 1]);
    if (h == LPP - 1) {
      dst[6 * CPL] = make_uint2((!st && finf) ? 1u : 0u, 0u);
      report(base + pt, st, first_bad, status);
    }
  }
  __syncthreads();
  if (cnt == PTS) {
    uint4* dst = (uint4*)((uint8_t*)out + base * ROUT);  // PTS * ROUT is a multiple of 16
    for (int k = t; k < PTS * ROUT / 16; k += BLK) {
      if (NT) st_stream(dst + k, slab[k]);
      else dst[k] = slab[k];
    }
  } else {  // ragged tail block: the slab ends on an 8-B boundary
    uint2* dst = (uint2*)out + base * (ROUT / 8);
    const uint2* s2 = (const uint2*)slab;
    for (int k = t; k < cnt * (ROUT / 8); k += BLK) dst[k] = s2[k];
  }
}

// DIRECT input, one coordinate per lane (NC lanes per point: G1 x | y, G2 x.c0 | x.c1 | y.c0 |
// y.c1): each lane reads its 48-B coordinate straight from HBM (three 16-B loads at the record
// stride, through the caches — the three loads of a wave cover its records together) and only the
// output goes through the LDS slab, so the block has one barrier instead of two. Same bytes and
// statuses as k_load (tools/microbench/loader_ceiling.hip verifies the bytes; the loader tests the
// statuses). G1 (k_load_direct<2, 128>) against the staged kernel on four round-6 boxes: 5.63 /
// 5.81 / 5.63 / 5.81 TB/s against 5.38 / 5.55 / 5.40 / 5.82 (profiles/r06b, r06d, r06e,
// r06f_loader_ceiling.txt, "DIN plain 128"); one round-5 box had it 2 % slower (r05i). With
// nontemporal loads it is slower everywhere: the loads of neighbouring lanes share cache lines.
// G2 (k_load_direct<4, 32>) against the staged k_load<4, 32>: 5.65-5.66 against 5.56-5.57 TB/s
// (profiles/r06h, r06i_loader_ceiling.txt). The loaders keep the SIMDs issuing VALU ~83 % of their
// cycles (profiles/r06n_loader_stalls.json), so VALU instructions cost bandwidth here: every lane
// converting (no zero-initialised results for a tail block's idle lanes), a branch for the rare
// zero-fill and the filtered conditional subtraction (words_to_ark_mont<true>) took G1 5.70-5.72 ->
// 5.81-5.87 and G2 5.57-5.59 -> 5.72-5.88 TB/s on one box (r06s_loader_ceiling.txt, bytes equal; the
// filter alone +0.1-3 %). A wave-uniform filter on the input range test measured slower (r06q).
// Status order is ark's: the first failing coordinate in x.c0, x.c1, y.c0, (flags), y.c1 order.
template <int NC, int PTS, bool FILTER = true>  // FILTER: words_to_ark_mont's (false: r06s's A side)
__global__ void __launch_bounds__(PTS * NC) k_load_direct(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                          uint64_t n, unsigned long long* __restrict__ first_bad,
                                                          uint8_t* __restrict__ status) {
  constexpr int BLK = PTS * NC, RIN = 48 * NC, ROUT = 48 * NC + 8;
  static_assert(NC == 2 || NC == 4, "G1 or G2");
  static_assert((PTS * ROUT) % 16 == 0 && BLK % 64 == 0, "slab alignment, whole waves");
  __shared__ uint4 slab[PTS * ROUT / 16];
  const uint64_t base = (uint64_t)blockIdx.x * PTS;
  const int cnt = (int)((n - base) < (uint64_t)PTS ? (n - base) : (uint64_t)PTS);
  const int t = threadIdx.x, pt = t / NC, h = t % NC;
  const bool last = h == NC - 1;  // the coordinate that carries the SWFlags
  // Every lane converts: the idle lanes of a ragged tail block re-read the block's last record and
  // write nothing, so no lane needs zero-initialised results (13 fewer VALU per lane).
  const bool live = pt < cnt;
  words c, res;
  load_le(c, in + (base + (live ? pt : cnt - 1)) * (RIN / 16) + 3 * h);
  const uint32_t yb = c[11] >> 24;
  const bool finf = last && (yb & 0x40u);
  int st = 0;
  if (last) {
    c[11] &= 0x3fffffffu;
    if ((yb & 0x80u) && finf) st = 6;  // both SWFlags: UnexpectedFlags, before y's last range check
  }
  if (!st && words_geq_p(c)) st = 3;
  words_to_ark_mont<FILTER>(res, c);
  // the point's status: the first failing coordinate's (lane order = ark's read order)
  int key = st ? (h << 8) | st : 0xffff;
#pragma unroll
  for (int m = 1; m < NC; m <<= 1) key = min(key, __shfl_xor(key, m));
  st = key == 0xffff ? 0 : key & 0xff;
  if (live) {
    uint2* dst = (uint2*)slab + pt * (ROUT / 8) + 6 * h;
#pragma unroll
    for (int j = 0; j < 6; j++) dst[j] = make_uint2(res[2 * j], res[2 * j + 1]);
    if (st)  // rare: a rejected point is zero-filled (a branch instead of 12 selects per lane)
#pragma unroll
      for (int j = 0; j < 6; j++) dst[j] = make_uint2(0, 0);
    if (last) {
      dst[6] = make_uint2((!st && finf) ? 1u : 0u, 0u);
      report(base + pt, st, first_bad, status);
    }
  }
  __syncthreads();
  if (cnt == PTS) {
    uint4* dst = (uint4*)((uint8_t*)out + base * ROUT);
    for (int k = t; k < PTS * ROUT / 16; k += BLK) st_stream(dst + k, slab[k]);
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
    // one coordinate per lane, direct input: 5.66-5.67 TB/s at 16 / 32 / 64-point blocks against
    // 5.55-5.59 for the staged lane-pair kernel in one-wave blocks (k_load<4, 32>, the product from
    // round 4 to 6: profiles/r06h_loader_ceiling.txt, same bytes)
    constexpr int P = 32;  // 128 lanes, 6.4 KB of output slab
    hipLaunchKernelGGL((k_load_direct<4, P>), dim3((unsigned)((n + P - 1) / P)), dim3(P * 4), 0, stream,
                       (const uint4*)d_in, (uint4*)d_out, n, d_first_bad, d_status);
  } else {
    constexpr int P = 128;  // one coordinate per lane: 256 lanes, 13.3 KB of output slab
    hipLaunchKernelGGL((k_load_direct<2, P>), dim3((unsigned)((n + P - 1) / P)), dim3(P * 2), 0, stream,
                       (const uint4*)d_in, (uint4*)d_out, n, d_first_bad, d_status);
  }
  return hipGetLastError();
}

}  // namespace kzgpot
