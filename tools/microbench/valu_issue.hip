// Per-opcode VALU issue cost on gfx950: SIMD cycles per wave64 instruction
// for the opcodes the codec kernels are made of, at 1, 2, 4 and 8 waves per SIMD, with 8
// independent chains per wave (throughput) and with one dependent chain (latency).
//
// Clock: every wave reads s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop, so
// the reported cycles are the cycles the SIMD actually ran, whatever the box's clock was.
// cycles per instruction per SIMD = (wave's loop cycles) / (instructions the W co-resident waves
// issued) — every wave of the grid is resident from start to end (grid = 256 CUs x W blocks of
// one wave per SIMD).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o bin/valu_issue valu_issue.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                                                 \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                   \
    }                                                                                            \
  } while (0)

enum Op {
  MAD64, MULLO, MULHI, ADD, SUB, ADDCO, ADDC, AND, XOR, LSHR, LSHL, LSHR64, LSHLADD64, LSHLADD, ADD3,
  ANDOR, OR3, CNDMASK, MOV, BFE, ALIGNBIT, MUL24, MULHI24, MAD24, FMA64, MIX_MAD_AND, MIX_MAD3_ADD,
  MIX_MAD_LSHR64, MIX_MAD_MULLO, NOPS
};
static const char* kName[NOPS] = {
    "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_add_u32", "v_sub_u32", "v_add_co_u32",
    "v_addc_co_u32", "v_and_b32", "v_xor_b32", "v_lshrrev_b32", "v_lshlrev_b32", "v_lshrrev_b64",
    "v_lshl_add_u64", "v_lshl_add_u32", "v_add3_u32", "v_and_or_b32", "v_or3_b32", "v_cndmask_b32",
    "v_mov_b32", "v_bfe_u32", "v_alignbit_b32", "v_mul_u32_u24", "v_mul_hi_u32_u24", "v_mad_u32_u24",
    "v_fma_f64", "mix 1 mad64 : 1 and", "mix 3 mad64 : 1 add", "mix 1 mad64 : 1 lshr64",
    "mix 1 mad64 : 1 mul_lo"};

template <int OP>
__device__ __forceinline__ void step(uint32_t& x, uint64_t& a, double& f, uint32_t y, uint64_t y64, double g,
                                     uint64_t smask) {
  if constexpr (OP == MAD64) {
    uint64_t cc;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a), "=s"(cc) : "v"(x), "v"(y));
  } else if constexpr (OP == MULLO) {
    asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == MULHI) {
    asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == ADD) {
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == SUB) {
    asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == ADDCO) {
    asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(y) : "vcc");
  } else if constexpr (OP == ADDC) {
    asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(y) : "vcc");
  } else if constexpr (OP == AND) {
    asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == XOR) {
    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == LSHR) {
    asm volatile("v_lshrrev_b32 %0, 5, %0" : "+v"(x));
  } else if constexpr (OP == LSHL) {
    asm volatile("v_lshlrev_b32 %0, 5, %0" : "+v"(x));
  } else if constexpr (OP == LSHR64) {
    asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(a));
  } else if constexpr (OP == LSHLADD64) {
    asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a) : "v"(y64));
  } else if constexpr (OP == LSHLADD) {
    asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == ADD3) {
    asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == ANDOR) {
    asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == OR3) {
    asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == CNDMASK) {
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(smask));
  } else if constexpr (OP == MOV) {
    asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(y));
  } else if constexpr (OP == BFE) {
    asm volatile("v_bfe_u32 %0, %0, 3, 28" : "+v"(x));
  } else if constexpr (OP == ALIGNBIT) {
    asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(y));
  } else if constexpr (OP == MUL24) {
    asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == MULHI24) {
    asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y));
  } else if constexpr (OP == MAD24) {
    asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x) : "v"(y));
  } else if constexpr (OP == FMA64) {
    asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(f) : "v"(g));
  } else if constexpr (OP == MIX_MAD_AND) {
    step<MAD64>(x, a, f, y, y64, g, smask);
    step<AND>(x, a, f, y, y64, g, smask);
  } else if constexpr (OP == MIX_MAD3_ADD) {
    step<MAD64>(x, a, f, y, y64, g, smask);
    step<MAD64>(x, a, f, y, y64, g, smask);
    step<MAD64>(x, a, f, y, y64, g, smask);
    step<ADD>(x, a, f, y, y64, g, smask);
  } else if constexpr (OP == MIX_MAD_LSHR64) {
    uint64_t cc;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a), "=s"(cc) : "v"(x), "v"(y));
    asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(a));
  } else if constexpr (OP == MIX_MAD_MULLO) {
    step<MAD64>(x, a, f, y, y64, g, smask);
    step<MULLO>(x, a, f, y, y64, g, smask);
  }
}
constexpr int ops_per_step(int op) { return op == MIX_MAD3_ADD ? 4 : (op >= MIX_MAD_AND ? 2 : 1); }

// CH independent chains, each advanced UNROLL times per loop iteration.
template <int OP, int CH>
__global__ __launch_bounds__(256) void kern(uint64_t* out, uint64_t* clk, int iters, uint32_t seed) {
  constexpr int UNROLL = 64 / CH;
  uint32_t x[CH];
  uint64_t a[CH];
  double f[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) {
    x[k] = seed * (threadIdx.x + 17 * k + 1);
    a[k] = ((uint64_t)x[k] << 20) ^ seed;
    f[k] = 1.0 + 1e-9 * x[k];
  }
  const uint32_t y = seed ^ blockIdx.x;
  const uint64_t y64 = (uint64_t)y * 3;
  const double g = 0.999999;
  const uint64_t smask = 0x5555555555555555ull ^ seed;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
#pragma unroll
      for (int k = 0; k < CH; k++) step<OP>(x[k], a[k], f[k], y, y64, g, smask);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; k++) s ^= x[k] ^ a[k] ^ (uint64_t)__double_as_longlong(f[k]);
  const int w = blockIdx.x * 4 + threadIdx.x / 64;
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) {
    clk[w * 4] = t1 - t0;
    clk[w * 4 + 1] = r1 - r0;
    clk[w * 4 + 2] = r0;
    clk[w * 4 + 3] = r1;
  }
}

using KernFn = void (*)(uint64_t*, uint64_t*, int, uint32_t);
template <int OP>
KernFn pick(int ch) {
  return ch == 1 ? (KernFn)kern<OP, 1>
                 : ch == 2 ? (KernFn)kern<OP, 2> : ch == 4 ? (KernFn)kern<OP, 4> : (KernFn)kern<OP, 8>;
}
template <int... OPS>
KernFn table_impl(int op, int ch, std::integer_sequence<int, OPS...>) {
  KernFn f = nullptr;
  ((op == OPS ? (f = pick<OPS>(ch), 0) : 0), ...);
  return f;
}
KernFn table(int op, int ch) { return table_impl(op, ch, std::make_integer_sequence<int, NOPS>{}); }

struct Res {
  double per_wave;  // each wave's own loop cycles / (its instructions x W): assumes W co-resident waves
  double chip;      // launch span (first wave start .. last wave end) x SIMDs / all instructions issued
  double mhz;
};
Res run(int op, int ch, int W, int cus, uint64_t* out, uint64_t* clk, std::vector<uint64_t>& h) {
  const int blocks = cus * W, iters = 1000;  // 256-thread blocks: one wave per SIMD each
  KernFn f = table(op, ch);
  hipLaunchKernelGGL(f, blocks, 256, 0, 0, out, clk, 16, 1u);  // warm
  hipLaunchKernelGGL(f, blocks, 256, 0, 0, out, clk, iters, 3u);
  CHECK(hipDeviceSynchronize());
  const int waves = blocks * 4;
  CHECK(hipMemcpy(h.data(), clk, (size_t)waves * 32, hipMemcpyDeviceToHost));
  double cyc = 0, rt = 0;
  uint64_t lo = ~0ull, hi = 0;
  for (int w = 0; w < waves; w++) {
    cyc += h[4 * w], rt += h[4 * w + 1];
    lo = std::min(lo, h[4 * w + 2]);
    hi = std::max(hi, h[4 * w + 3]);
  }
  Res r;
  r.mhz = cyc / rt * 100.0;
  cyc /= waves;
  const double instrs = (double)iters * 64 * ops_per_step(op);
  r.per_wave = cyc / (instrs * W);
  r.chip = (double)(hi - lo) * (r.mhz / 100.0) * (cus * 4) / (instrs * waves);
  return r;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs=%d\n", prop.gcnArchName, cus);
  printf("SIMD cycles per wave64 VALU instruction, shown as chip / wave:\n"
         "  chip = launch span (first wave start .. last wave end, s_memrealtime) x shader clock\n"
         "         (s_memtime / s_memrealtime) x SIMDs / instructions issued by the whole grid;\n"
         "  wave = a wave's own loop cycles / (its instructions x W) (assumes all W waves co-resident).\n"
         "W = waves per SIMD (grid = CUs x W blocks of 256 threads); chains = independent dependency chains per wave.\n");
  const int maxW = 8;
  uint64_t *out, *clk;
  CHECK(hipMalloc(&out, (size_t)cus * maxW * 256 * 8));
  CHECK(hipMalloc(&clk, (size_t)cus * maxW * 4 * 32));
  std::vector<uint64_t> h((size_t)cus * maxW * 4 * 4);
  const int Ws[6] = {1, 2, 3, 4, 6, 8};
  const int chs[4] = {1, 2, 4, 8};
  for (int op = 0; op < NOPS; op++) {
    printf("\n%-22s        W=1         W=2         W=3         W=4         W=6         W=8\n", kName[op]);
    for (int ci = 0; ci < 4; ci++) {
      const bool all_chains = op == MAD64 || op == ADD || op == MIX_MAD_AND || op == MIX_MAD3_ADD;
      if (!all_chains && chs[ci] != 1 && chs[ci] != 8) continue;
      printf("  chains=%d         ", chs[ci]);
      double mhz = 0;
      for (int wi = 0; wi < 6; wi++) {
        const Res r = run(op, chs[ci], Ws[wi], cus, out, clk, h);
        printf(" %5.2f/%5.2f", r.chip, r.per_wave);
        mhz += r.mhz / 6;
      }
      printf("  %4.0f MHz\n", mhz);
    }
  }
  return 0;
}
