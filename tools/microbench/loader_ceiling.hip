// Ceiling of the loader's memory pattern: k_load<G1> reads 96 B and writes
// 104 B per point (ark bytes -> in-memory GroupAffine), staged through LDS so every global access is
// a contiguous 16-B-per-lane sweep. How fast can that PATTERN go on this HBM, without the Fp work?
//
//   copy16        : plain 16-B-per-lane copy of the same input bytes (the guide's float4 copy)
//   slab          : k_load's exact staging without the arithmetic — slab in, per-lane 96-B record
//                   read at a 96-B LDS stride, 104-B record written back at a 104-B stride, slab out
//   slab_nt_st    : slab with nontemporal (streaming) global stores
//   slab_nt       : slab with nontemporal loads and stores
//   slab_glds_nt  : slab whose input sweep is global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip)
//                   + nontemporal stores
//   product G1/G2 : the product kernels (kzgpot::launch_load: k_load_direct<2, 128> / <4, 32> since
//                   round 6), for the same bytes; "k_load 1c/l 128" / "k_load<G2> 32" are the round-5
//                   products (staged in and out)
//   k_load_pipe   : an experiment: a resident grid (x f/4 of the occupancy-limited block count)
//                   walks the slabs grid-stride, prefetching the next slab's input into registers
//                   while it converts and stores the current one. Slower than letting the hardware
//                   keep ~8 independent blocks per CU in flight (4.9 vs 5.55 TB/s)
// Every variant moves 96 + 104 B per point for 2^27 points (12.9 GB read + 14.0 GB written; copy16
// moves 96 + 96). Reported: ms per launch (hipEvent, mean of 10 after 2 warm-ups) and TB/s of
// algorithmic bytes.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bin/loader_ceiling loader_ceiling.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../kzg-setup-powersoftau_amd/csrc/load_kernels.hip"

// The same per-point work as k_load, software-pipelined: a grid of resident blocks walks the
// slabs grid-stride, and each block issues the NEXT slab's input loads (into registers, PER per
// lane) before it converts and stores the current one, so the input latency hides behind the
// block's own compute and store sweep instead of only behind other blocks'.
namespace kzgpot {
// EXPERIMENT (not in the product; measured slower, profiles/r03_loader_ceiling.txt):
template <int NC, int PTS, int CPL = 2>
__global__ void __launch_bounds__(PTS * NC / CPL) k_load_pipe(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                              uint64_t n, unsigned long long* __restrict__ first_bad,
                                                              uint8_t* __restrict__ status) {
  constexpr int LPP = NC / CPL, BLK = PTS * LPP;
  constexpr int RIN = 48 * NC, ROUT = 48 * NC + 8;
  constexpr int NIN16 = PTS * RIN / 16, PER = (NIN16 + BLK - 1) / BLK;
  static_assert(LPP == 1 || LPP == 2, "a point is one lane or a lane pair");
  static_assert(RIN % 16 == 0 && (PTS * ROUT) % 16 == 0 && ROUT % 8 == 0, "slab alignment");
  __shared__ uint4 slab[PTS * ROUT / 16];
  const uint64_t nslabs = (n + PTS - 1) / PTS;
  const int t = threadIdx.x;
  const int pt = t / LPP, h = t % LPP;
  uint4 pre[PER];
  auto fetch = [&](uint64_t sl) {
    const uint64_t b = sl * PTS;
    const int c = (int)((n - b) < (uint64_t)PTS ? (n - b) : (uint64_t)PTS);
    const uint4* src = in + b * (RIN / 16);
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int k = t + q * BLK;
      if (k < c * (RIN / 16)) pre[q] = ld_stream(src + k);
    }
  };
  uint64_t sl = blockIdx.x;
  if (sl < nslabs) fetch(sl);
  for (; sl < nslabs; sl += gridDim.x) {
    const uint64_t base = sl * PTS;
    const int cnt = (int)((n - base) < (uint64_t)PTS ? (n - base) : (uint64_t)PTS);
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int k = t + q * BLK;
      if (k < cnt * (RIN / 16)) slab[k] = pre[q];
    }
    __syncthreads();
    if (sl + gridDim.x < nslabs) fetch(sl + gridDim.x);  // in flight during the work below

    int st = 0;
    bool finf = false;
    words res[CPL];
    if (pt < cnt) {
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
    if (LPP == 2) {
      const int other = __shfl_xor(st, 1);
      st = h == 0 ? (st ? st : other) : (other ? other : st);
    }
    __syncthreads();
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
      uint4* dst = (uint4*)((uint8_t*)out + base * ROUT);
      for (int k = t; k < PTS * ROUT / 16; k += BLK) st_stream(dst + k, slab[k]);
    } else {
      uint2* dst = (uint2*)out + base * (ROUT / 8);
      const uint2* s2 = (const uint2*)slab;
      for (int k = t; k < cnt * (ROUT / 8); k += BLK) dst[k] = s2[k];
    }
    __syncthreads();  // the slab is read out before the next slab's input overwrites it
  }
}
// k_load with DIRECT input — each lane reads its own coordinates straight from global memory (48-B
// pieces at the record stride) instead of from a staged input slab; the slab stages only the
// output, and the block's first barrier goes away. G2 (two coordinates per lane): 3.70-3.83 TB/s
// against 5.56-5.62 for the staged kernel (r05i, r06*). G1 with plain loads: faster than the staged
// kernel on three of four round-6 boxes (r06b/d/e: 5.63-5.81 against 5.38-5.55 TB/s, equal on
// r06f), slower on r05i's (5.48 / 5.61) — the product G1 loader since round 6 (k_load_direct<2, 128> in
// load_kernels.hip); with nontemporal loads slower everywhere.
template <int NC, int PTS, bool NT, int CPL>
__global__ void __launch_bounds__(PTS * NC / CPL) k_load_din(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                             uint64_t n, unsigned long long* __restrict__ first_bad,
                                                             uint8_t* /* status: not kept */) {
  constexpr int LPP = NC / CPL, BLK = PTS * LPP;
  constexpr int RIN = 48 * NC, ROUT = 48 * NC + 8;
  __shared__ uint4 slab[PTS * ROUT / 16];
  const uint64_t base = (uint64_t)blockIdx.x * PTS;
  const int cnt = (int)((n - base) < (uint64_t)PTS ? (n - base) : (uint64_t)PTS);
  const int t = threadIdx.x, pt = t / LPP, h = t % LPP;
  int st = 0;
  bool finf = false;
  words res[CPL];
  if (pt < cnt) {
    const uint4* rec = in + (base + pt) * (RIN / 16) + 3 * CPL * h;
    const bool last = h == LPP - 1;
    words c[CPL];
#pragma unroll
    for (int k = 0; k < CPL; k++) {
      uint4 a, b, d;
      if (NT) a = ld_stream(rec + 3 * k), b = ld_stream(rec + 3 * k + 1), d = ld_stream(rec + 3 * k + 2);
      else a = rec[3 * k], b = rec[3 * k + 1], d = rec[3 * k + 2];
      c[k][0] = a.x, c[k][1] = a.y, c[k][2] = a.z, c[k][3] = a.w, c[k][4] = b.x, c[k][5] = b.y;
      c[k][6] = b.z, c[k][7] = b.w, c[k][8] = d.x, c[k][9] = d.y, c[k][10] = d.z, c[k][11] = d.w;
    }
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
  if (LPP == 2) {
    const int other = __shfl_xor(st, 1);
    st = h == 0 ? (st ? st : other) : (other ? other : st);
  }
  if (pt < cnt) {
    uint2* dst = (uint2*)slab + pt * (ROUT / 8) + 6 * CPL * h;
#pragma unroll
    for (int k = 0; k < CPL; k++)
#pragma unroll
      for (int j = 0; j < 6; j++) dst[6 * k + j] = st ? make_uint2(0, 0) : make_uint2(res[k][2 * j], res[k][2 * j + 1]);
    if (h == LPP - 1) {
      dst[6 * CPL] = make_uint2((!st && finf) ? 1u : 0u, 0u);
      report(base + pt, st, first_bad, nullptr);
    }
  }
  __syncthreads();
  uint4* dst = (uint4*)((uint8_t*)out + base * ROUT);  // full blocks only (n is a multiple of PTS here)
  for (int k = t; k < PTS * ROUT / 16; k += BLK) st_stream(dst + k, slab[k]);
}

// k_load_direct with DIRECT OUTPUT too (round 6 experiment): no LDS slab and no barrier — each lane
// writes its converted 48-B coordinate straight to its place in the output record (8-B aligned at
// the 104- / 200-B record stride), the flags lane also the 8-B infinity word, and the L2 merges
// neighbouring lanes' pieces into whole lines before write-back. ST 0: plain 8-B stores; 1:
// nontemporal 8-B stores; 2: 16-B stores at 4-B alignment (unaligned-access mode). The compiler
// emits three 16-B stores per lane in every case. Measured (profiles/r06m_loader_ceiling.txt, bytes
// equal): G1 4.69 TB/s, G2 4.40 (4.90 at 64-point blocks) against 5.66 / 5.52 for the product on
// the same box; with nontemporal stores 1.9-2.3 TB/s. Staging the output pays: NOT in the product.
struct __attribute__((packed, aligned(4))) u4a {
  uint32_t x, y, z, w;
};
template <int NC, int PTS, int ST>
__global__ void __launch_bounds__(PTS * NC) k_load_dd(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n,
                                                      unsigned long long* __restrict__ first_bad, uint8_t* status) {
  constexpr int RIN = 48 * NC, ROUT = 48 * NC + 8;
  const uint64_t base = (uint64_t)blockIdx.x * PTS;
  const int t = threadIdx.x, pt = t / NC, h = t % NC;
  const bool last = h == NC - 1, live = base + pt < n;
  int st = 0;
  bool finf = false;
  words res;
  if (live) {
    words c;
    load_le(c, in + (base + pt) * (RIN / 16) + 3 * h);
    const uint32_t yb = c[11] >> 24;
    finf = last && (yb & 0x40u);
    if (last) {
      c[11] &= 0x3fffffffu;
      if ((yb & 0x80u) && finf) st = 6;
    }
    if (!st && words_geq_p(c)) st = 3;
    words_to_ark_mont(res, c);
  }
  int key = st ? (h << 8) | st : 0xffff;
#pragma unroll
  for (int m = 1; m < NC; m <<= 1) key = min(key, __shfl_xor(key, m));
  st = key == 0xffff ? 0 : key & 0xff;
  if (!live) return;
  uint8_t* rec = (uint8_t*)out + (base + pt) * ROUT + 48 * h;
  if (st)
#pragma unroll
    for (int k = 0; k < 12; k++) res[k] = 0;
  if (ST == 2) {
    u4a* d = (u4a*)rec;
#pragma unroll
    for (int j = 0; j < 3; j++) d[j] = u4a{res[4 * j], res[4 * j + 1], res[4 * j + 2], res[4 * j + 3]};
  } else {
    uint2* d = (uint2*)rec;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const uint2 v = make_uint2(res[2 * j], res[2 * j + 1]);
      if (ST == 1) __builtin_nontemporal_store(*(const uint64_t*)&v, (uint64_t*)(d + j));
      else d[j] = v;
    }
  }
  if (last) {
    *(uint2*)(rec + 48) = make_uint2((!st && finf) ? 1u : 0u, 0u);
    report(base + pt, st, first_bad, status);
  }
}

// k_load_direct as it ran in r06h-r06n (the A side of the r06o/r06q changes): tail-block lanes
// skipped the conversion (so the compiler zero-initialised their results), a rejected point was
// zero-filled by 12 selects per lane instead of a branch, and the range test and the conversion's
// conditional subtraction ran in every lane (no wave-uniform filter).
template <int NC, int PTS>
__global__ void __launch_bounds__(PTS * NC) k_load_direct_r06n(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                               uint64_t n, unsigned long long* __restrict__ first_bad,
                                                               uint8_t* __restrict__ status) {
  constexpr int BLK = PTS * NC, RIN = 48 * NC, ROUT = 48 * NC + 8;
  __shared__ uint4 slab[PTS * ROUT / 16];
  const uint64_t base = (uint64_t)blockIdx.x * PTS;
  const int cnt = (int)((n - base) < (uint64_t)PTS ? (n - base) : (uint64_t)PTS);
  const int t = threadIdx.x, pt = t / NC, h = t % NC;
  const bool last = h == NC - 1;
  int st = 0;
  bool finf = false;
  words res;
  if (pt < cnt) {
    words c;
    load_le(c, in + (base + pt) * (RIN / 16) + 3 * h);
    const uint32_t yb = c[11] >> 24;
    finf = last && (yb & 0x40u);
    if (last) {
      c[11] &= 0x3fffffffu;
      if ((yb & 0x80u) && finf) st = 6;
    }
    if (!st && words_geq_p(c)) st = 3;
    words_to_ark_mont<false>(res, c);
  }
  int key = st ? (h << 8) | st : 0xffff;
#pragma unroll
  for (int m = 1; m < NC; m <<= 1) key = min(key, __shfl_xor(key, m));
  st = key == 0xffff ? 0 : key & 0xff;
  if (pt < cnt) {
    uint2* dst = (uint2*)slab + pt * (ROUT / 8) + 6 * h;
#pragma unroll
    for (int j = 0; j < 6; j++) dst[j] = st ? make_uint2(0, 0) : make_uint2(res[2 * j], res[2 * j + 1]);
    if (last) {
      dst[6] = make_uint2((!st && finf) ? 1u : 0u, 0u);
      report(base + pt, st, first_bad, status);
    }
  }
  __syncthreads();
  if (cnt == PTS) {
    uint4* dst = (uint4*)((uint8_t*)out + base * ROUT);
    for (int k = t; k < PTS * ROUT / 16; k += BLK) st_stream(dst + k, slab[k]);
  } else {
    uint2* dst = (uint2*)out + base * (ROUT / 8);
    const uint2* s2 = (const uint2*)slab;
    for (int k = t; k < cnt * (ROUT / 8); k += BLK) dst[k] = s2[k];
  }
}
}  // namespace kzgpot

#define CHECK(x)                                                                                 \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                   \
    }                                                                                            \
  } while (0)

constexpr int BLK = 256;
typedef uint32_t u4v __attribute__((ext_vector_type(4)));  // the nontemporal builtins need a vector type
typedef __attribute__((address_space(3))) void lds_void;
constexpr int RIN16 = 6, ROUT8 = 13, ROUT16X = 13;  // 96 B = 6 x 16; 104 B = 13 x 8

__global__ void __launch_bounds__(256) k_copy16(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) out[i] = in[i];
}

template <bool NT_LD, bool NT_ST, bool GLDS>
__global__ void __launch_bounds__(BLK) k_slab(const uint4* __restrict__ in, uint4* __restrict__ out) {
  __shared__ uint4 slab[BLK * ROUT8 / 2];
  const int t = threadIdx.x;
  const uint4* src = in + (uint64_t)blockIdx.x * BLK * RIN16;
  if constexpr (GLDS) {
    // one global_load_lds_dwordx4 per wave writes 64 x 16 B contiguously at the wave's LDS base
    const int w = t >> 6;
#pragma unroll
    for (int k = 0; k < RIN16; k++) {
      const int chunk = k * (BLK / 64) + w;  // 1 KiB chunks of the 24 KiB slab
      __builtin_amdgcn_global_load_lds((const void*)(src + chunk * 64 + (t & 63)), (lds_void*)(slab + chunk * 64),
                                       16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int k = t; k < BLK * RIN16; k += BLK) {
      if (NT_LD) {
        const u4v v = __builtin_nontemporal_load((const u4v*)(src + k));
        slab[k] = make_uint4(v.x, v.y, v.z, v.w);
      } else {
        slab[k] = src[k];
      }
    }
  }
  __syncthreads();
  uint4 r[RIN16];
#pragma unroll
  for (int j = 0; j < RIN16; j++) r[j] = slab[t * RIN16 + j];
  __syncthreads();
  uint2* d = (uint2*)slab + t * ROUT8;
#pragma unroll
  for (int j = 0; j < RIN16; j++) {
    d[2 * j] = make_uint2(r[j].x ^ 1u, r[j].y);  // ^1: the bytes change, as the conversion changes them
    d[2 * j + 1] = make_uint2(r[j].z, r[j].w);
  }
  d[12] = make_uint2(0, 0);
  __syncthreads();
  uint4* dst = out + (uint64_t)blockIdx.x * BLK * ROUT8 / 2;
  for (int k = t; k < BLK * ROUT8 / 2; k += BLK) {
    if (NT_ST) {
      const uint4 v = slab[k];
      __builtin_nontemporal_store((u4v){v.x, v.y, v.z, v.w}, (u4v*)(dst + k));
    } else {
      dst[k] = slab[k];
    }
  }
}

// random canonical ark records: every word pseudo-random, each coordinate's top word < 2^28 (value
// < 2^380 < p, flag bits clear), so k_load converts real data (all-zero input toggles fewer bits)
__global__ void k_fill(uint32_t* w, uint64_t nw) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nw) return;
  uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  uint32_t v = (uint32_t)(z ^ (z >> 31));
  if (i % 12 == 11) v &= 0x0fffffffu;
  w[i] = v;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 27;
  const uint64_t n = 1ull << lg;
  uint4 *in, *out;
  unsigned long long* key;
  CHECK(hipMalloc(&in, n * 96));
  CHECK(hipMalloc(&out, n * 104));
  CHECK(hipMalloc(&key, 8));
  const bool zero = argc > 2 && argv[2][0] == 'z';
  if (zero) {
    CHECK(hipMemset(in, 0, n * 96));
  } else {
    hipLaunchKernelGGL(k_fill, dim3((unsigned)(n * 24 / 256)), dim3(256), 0, 0, (uint32_t*)in, n * 24);
  }
  printf("input: %s, 2^%d points\n", zero ? "all zero" : "random canonical records", lg);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double rw = (96.0 + 104.0) * n;
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 2; i++) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < 10; i++) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    printf("%-16s %8.3f ms  %6.3f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  const unsigned gs = (unsigned)(n / BLK);
  {  // the DIN variants must write exactly the product kernel's bytes (G1 over n, G2 over n / 2)
    const size_t ob = n * 104;
    uint8_t* want = (uint8_t*)malloc(ob);
    uint8_t* got = (uint8_t*)malloc(ob);
    auto cmp = [&](const char* name, size_t nb, auto a, auto b) {  // the first nb output bytes
      CHECK(hipMemset(out, 0xA5, ob));
      a();
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(want, out, ob, hipMemcpyDeviceToHost));
      CHECK(hipMemset(out, 0x5A, ob));
      b();
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(got, out, ob, hipMemcpyDeviceToHost));
      printf("verify %-14s %s\n", name, memcmp(want, got, nb) == 0 ? "equal" : "DIFFERENT");
      // where they differ: the first differing byte's record and field, and
      // how many records differ
      const size_t rec = nb == n * 104 ? 104 : 200;
      size_t first = nb, nrec = 0;
      for (size_t r = 0; r < nb / rec; r++) {
        if (memcmp(want + r * rec, got + r * rec, rec) == 0) continue;
        if (!nrec)
          for (size_t b = 0; b < rec; b++)
            if (want[r * rec + b] != got[r * rec + b]) {
              first = r * rec + b;
              break;
            }
        nrec++;
      }
      if (nrec) {
        const size_t r = first / rec, b = first % rec;
        printf("  first difference: record %zu (block %zu of the variant's grid), byte %zu of %zu (%s), "
               "product %02x variant %02x; %zu of %zu records differ\n",
               r, r / (rec == 104 ? 128 : 32), b, rec, b < rec - 8 ? "coordinate" : "infinity flag / padding",
               want[first], got[first], nrec, nb / rec);
      }
    };
    cmp("staged (G1)", n * 104, [&] { CHECK(kzgpot::launch_load(false, in, out, n, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load<2, 128, true, 1>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n,
                         key, nullptr);
    });
    cmp("DIN 128 (G1)", n * 104, [&] { CHECK(kzgpot::launch_load(false, in, out, n, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_din<2, 128, true, 1>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out,
                         n, key, nullptr);
    });
    cmp("staged 32 (G2)", n / 2 * 200, [&] { CHECK(kzgpot::launch_load(true, in, out, n / 2, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load<4, 32>), dim3((unsigned)(n / 64)), dim3(64), 0, 0, in, out, n / 2, key, nullptr);
    });
    cmp("DIN 32 (G2)", n / 2 * 200, [&] { CHECK(kzgpot::launch_load(true, in, out, n / 2, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_din<4, 32, true, 2>), dim3((unsigned)(n / 64)), dim3(64), 0, 0, in, out,
                         n / 2, key, nullptr);
    });
    cmp("DD 128 (G1)", n * 104, [&] { CHECK(kzgpot::launch_load(false, in, out, n, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_dd<2, 128, 0>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n, key,
                         nullptr);
    });
    cmp("DD16 128 (G1)", n * 104, [&] { CHECK(kzgpot::launch_load(false, in, out, n, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_dd<2, 128, 2>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n, key,
                         nullptr);
    });
    cmp("DD 32 (G2)", n / 2 * 200, [&] { CHECK(kzgpot::launch_load(true, in, out, n / 2, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_dd<4, 32, 0>), dim3((unsigned)(n / 64)), dim3(128), 0, 0, in, out, n / 2, key,
                         nullptr);
    });
    cmp("DD16 32 (G2)", n / 2 * 200, [&] { CHECK(kzgpot::launch_load(true, in, out, n / 2, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_dd<4, 32, 2>), dim3((unsigned)(n / 64)), dim3(128), 0, 0, in, out, n / 2, key,
                         nullptr);
    });
    cmp("r06n direct (G1)", n * 104, [&] { CHECK(kzgpot::launch_load(false, in, out, n, key, nullptr, 0)); }, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_direct_r06n<2, 128>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n,
                         key, nullptr);
    });
    free(want);
    free(got);
  }
  for (int rep = 0; rep < 2; rep++) {
  printf("-- pass %d\n", rep);
  run("copy16", 192.0 * n, [&] { hipLaunchKernelGGL(k_copy16, dim3((unsigned)(n * 6 / 256)), dim3(256), 0, 0, in, out, n * 6); });
  run("slab", rw, [&] { hipLaunchKernelGGL((k_slab<false, false, false>), dim3(gs), dim3(BLK), 0, 0, in, out); });
  run("slab_nt_st", rw, [&] { hipLaunchKernelGGL((k_slab<false, true, false>), dim3(gs), dim3(BLK), 0, 0, in, out); });
  run("slab_nt", rw, [&] { hipLaunchKernelGGL((k_slab<true, true, false>), dim3(gs), dim3(BLK), 0, 0, in, out); });
  run("slab_glds_nt", rw, [&] { hipLaunchKernelGGL((k_slab<false, true, true>), dim3(gs), dim3(BLK), 0, 0, in, out); });
  run("k_load_plain", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load<2, 256, false>), dim3(gs), dim3(256), 0, 0, in, out, n, key, nullptr);
  });
  // the product G1 loader: k_load_direct<2, 128> since round 6 (the round-5 product, staged in and out, is
  // "k_load 1c/l 128" below)
  run("product G1 (direct)", rw, [&] { CHECK(kzgpot::launch_load(false, in, out, n, key, nullptr, 0)); });
  run("direct G1 r06n", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_direct_r06n<2, 128>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n, key,
                       nullptr);
  });
  run("direct G1 nofilter", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_direct<2, 128, false>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n,
                       key, nullptr);
  });
  run("product G1 (again)", rw, [&] { CHECK(kzgpot::launch_load(false, in, out, n, key, nullptr, 0)); });
  // direct output (no slab): plain / nontemporal 8-B stores, 16-B stores at 4-B alignment
  run("DD G1 128 st8", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<2, 128, 0>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n, key, nullptr);
  });
  run("DD G1 128 nt8", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<2, 128, 1>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n, key, nullptr);
  });
  run("DD G1 128 st16", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<2, 128, 2>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n, key, nullptr);
  });
  run("DD G1 32 st8", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<2, 32, 0>), dim3((unsigned)(n / 32)), dim3(64), 0, 0, in, out, n, key, nullptr);
  });
  run("k_load 1c/l 128", rw, [&] {  // one coordinate per lane: 128 points = 256 lanes per block
    hipLaunchKernelGGL((kzgpot::k_load<2, 128, true, 1>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n, key,
                       nullptr);
  });
  run("k_load 1c/l 256", rw, [&] {  // 256 points = 512 lanes per block
    hipLaunchKernelGGL((kzgpot::k_load<2, 256, true, 1>), dim3((unsigned)(n / 256)), dim3(512), 0, 0, in, out, n, key,
                       nullptr);
  });
  // smaller blocks: fewer waves meet at each block barrier (32 points = one wave, 64 = two)
  run("k_load 1c/l 32", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load<2, 32, true, 1>), dim3((unsigned)(n / 32)), dim3(64), 0, 0, in, out, n, key,
                       nullptr);
  });
  run("k_load 1c/l 64", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load<2, 64, true, 1>), dim3((unsigned)(n / 64)), dim3(128), 0, 0, in, out, n, key,
                       nullptr);
  });
  // direct input (DIN): lanes read their coordinates straight from global memory, the slab stages
  // only the output, one block barrier instead of two
  run("k_load DIN 128", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_din<2, 128, true, 1>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n,
                       key, nullptr);
  });
  run("k_load DIN 64", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_din<2, 64, true, 1>), dim3((unsigned)(n / 64)), dim3(128), 0, 0, in, out, n,
                       key, nullptr);
  });
  run("k_load DIN 32", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_din<2, 32, true, 1>), dim3((unsigned)(n / 32)), dim3(64), 0, 0, in, out, n, key,
                       nullptr);
  });
  run("k_load DIN plain 128", rw, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_din<2, 128, false, 1>), dim3((unsigned)(n / 128)), dim3(256), 0, 0, in, out, n,
                       key, nullptr);
  });
  run("k_load 2c/l 128", rw, [&] {  // one lane per point, 128 points per block
    hipLaunchKernelGGL((kzgpot::k_load<2, 128, true, 2>), dim3((unsigned)(n / 128)), dim3(128), 0, 0, in, out, n, key,
                       nullptr);
  });
  // software-pipelined loader (k_load_pipe): a resident grid walks the slabs grid-stride and
  // prefetches the next slab's input while it converts and stores the current one
  int cus = 0, occ1 = 0, occ2 = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, kzgpot::k_load_pipe<2, 128, 1>, 256, 0));
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, kzgpot::k_load_pipe<4, 128, 2>, 256, 0));
  if (rep == 0) printf("k_load_pipe: %d CUs, %d / %d resident blocks per CU (G1 / G2)\n", cus, occ1, occ2);
  for (int f = 1; f <= 4; f *= 2) {
    char nm[32];
    snprintf(nm, sizeof nm, "k_load_pipe x%d/4", f);
    const unsigned g = (unsigned)(cus * occ1 * f / 4);
    run(nm, rw, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_pipe<2, 128, 1>), dim3(g), dim3(256), 0, 0, in, out, n, key, nullptr);
    });
  }
  // G2: 192 B in + 200 B out per point, half the points
  const uint64_t n2 = n / 2;
  for (int f = 2; f <= 4; f *= 2) {
    char nm[32];
    snprintf(nm, sizeof nm, "k_load_pipe<G2> x%d/4", f);
    const unsigned g = (unsigned)(cus * occ2 * f / 4);
    run(nm, (192.0 + 200.0) * n2, [&] {
      hipLaunchKernelGGL((kzgpot::k_load_pipe<4, 128, 2>), dim3(g), dim3(256), 0, 0, in, out, n2, key, nullptr);
    });
  }
  run("product G2 (direct)", (192.0 + 200.0) * n2, [&] { CHECK(kzgpot::launch_load(true, in, out, n2, key, nullptr, 0)); });
  run("direct G2 r06n", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_direct_r06n<4, 32>), dim3((unsigned)(n2 / 32)), dim3(128), 0, 0, in, out, n2, key,
                       nullptr);
  });
  run("direct G2 nofilter", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_direct<4, 32, false>), dim3((unsigned)(n2 / 32)), dim3(128), 0, 0, in, out, n2,
                       key, nullptr);
  });
  run("product G2 (again)", (192.0 + 200.0) * n2, [&] { CHECK(kzgpot::launch_load(true, in, out, n2, key, nullptr, 0)); });
  run("DD G2 32 st8", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<4, 32, 0>), dim3((unsigned)(n2 / 32)), dim3(128), 0, 0, in, out, n2, key, nullptr);
  });
  run("DD G2 32 nt8", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<4, 32, 1>), dim3((unsigned)(n2 / 32)), dim3(128), 0, 0, in, out, n2, key, nullptr);
  });
  run("DD G2 32 st16", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<4, 32, 2>), dim3((unsigned)(n2 / 32)), dim3(128), 0, 0, in, out, n2, key, nullptr);
  });
  run("DD G2 64 st8", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_dd<4, 64, 0>), dim3((unsigned)(n2 / 64)), dim3(256), 0, 0, in, out, n2, key, nullptr);
  });
  run("k_load<G2> 32", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load<4, 32, true, 2>), dim3((unsigned)(n2 / 32)), dim3(64), 0, 0, in, out, n2, key,
                       nullptr);
  });
  run("k_load<G2> 64", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load<4, 64, true, 2>), dim3((unsigned)(n2 / 64)), dim3(128), 0, 0, in, out, n2, key,
                       nullptr);
  });
  run("k_load<G2> DIN 32", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_din<4, 32, true, 2>), dim3((unsigned)(n2 / 32)), dim3(64), 0, 0, in, out, n2,
                       key, nullptr);
  });
  run("k_load<G2> DIN 64", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_din<4, 64, true, 2>), dim3((unsigned)(n2 / 64)), dim3(128), 0, 0, in, out, n2,
                       key, nullptr);
  });
  // one coordinate per lane, direct input (k_load_direct<4, PTS>: 4 lanes per point)
  run("k_load<G2> direct 16", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_direct<4, 16>), dim3((unsigned)(n2 / 16)), dim3(64), 0, 0, in, out, n2, key,
                       nullptr);
  });
  run("k_load<G2> direct 32", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_direct<4, 32>), dim3((unsigned)(n2 / 32)), dim3(128), 0, 0, in, out, n2, key,
                       nullptr);
  });
  run("k_load<G2> direct 64", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load_direct<4, 64>), dim3((unsigned)(n2 / 64)), dim3(256), 0, 0, in, out, n2, key,
                       nullptr);
  });
  run("k_load<G2>plain", (192.0 + 200.0) * n2, [&] {
    hipLaunchKernelGGL((kzgpot::k_load<4, 128, false>), dim3((unsigned)(n2 / 128)), dim3(256), 0, 0, in, out, n2, key,
                       nullptr);
  });
  }
  CHECK(hipGetLastError());
  return 0;
}
