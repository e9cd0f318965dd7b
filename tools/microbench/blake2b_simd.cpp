// BLAKE2b-512 compression variants on one core: scalar (csrc/blake2b.cpp's form), AVX2 and
// AVX-512VL (vprorq rotations). Build: g++ -O3 -std=c++17 blake2b_simd.cpp -o blake2b_simd
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <vector>

static const uint64_t IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                               0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                               0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
static const uint8_t SG[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void comp_scalar(uint64_t h[8], const uint8_t* blk, uint64_t t, bool last) {
  uint64_t m[16], v[16];
  memcpy(m, blk, 128);
  for (int i = 0; i < 8; i++) v[i] = h[i], v[i + 8] = IV[i];
  v[12] ^= t;
  if (last) v[14] = ~v[14];
#define G(a, b, c, d, x, y) a = a + b + x; d = rotr(d ^ a, 32); c = c + d; b = rotr(b ^ c, 24); \
  a = a + b + y; d = rotr(d ^ a, 16); c = c + d; b = rotr(b ^ c, 63);
#pragma GCC unroll 12
  for (int r = 0; r < 12; r++) {
    const uint8_t* s = SG[r];
    G(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]); G(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
    G(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]); G(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
    G(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]); G(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
    G(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]); G(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
  }
#undef G
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

template <bool AVX512>
__attribute__((target("avx2,avx512f,avx512vl"))) static void comp_vec(uint64_t h[8], const uint8_t* blk, uint64_t t,
                                                                      bool last) {
  uint64_t m[16];
  memcpy(m, blk, 128);
  const __m256i r16 = _mm256_setr_epi8(2, 3, 4, 5, 6, 7, 0, 1, 10, 11, 12, 13, 14, 15, 8, 9, 2, 3, 4, 5, 6, 7, 0, 1,
                                       10, 11, 12, 13, 14, 15, 8, 9);
  const __m256i r24 = _mm256_setr_epi8(3, 4, 5, 6, 7, 0, 1, 2, 11, 12, 13, 14, 15, 8, 9, 10, 3, 4, 5, 6, 7, 0, 1, 2,
                                       11, 12, 13, 14, 15, 8, 9, 10);
  __m256i a = _mm256_loadu_si256((const __m256i*)h), b = _mm256_loadu_si256((const __m256i*)(h + 4));
  __m256i c = _mm256_loadu_si256((const __m256i*)IV);
  __m256i d = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(IV + 4)),
                               _mm256_setr_epi64x((long long)t, 0, last ? -1ll : 0ll, 0));
  const __m256i a0 = a, b0 = b;
#define ROT(x, n, sh) (AVX512 ? _mm256_ror_epi64(x, n) : (sh))
#define G4(x, y)                                                                                 \
  a = _mm256_add_epi64(_mm256_add_epi64(a, b), x);                                               \
  d = _mm256_xor_si256(d, a); d = ROT(d, 32, _mm256_shuffle_epi32(d, _MM_SHUFFLE(2, 3, 0, 1)));  \
  c = _mm256_add_epi64(c, d);                                                                    \
  b = _mm256_xor_si256(b, c); b = ROT(b, 24, _mm256_shuffle_epi8(b, r24));                       \
  a = _mm256_add_epi64(_mm256_add_epi64(a, b), y);                                               \
  d = _mm256_xor_si256(d, a); d = ROT(d, 16, _mm256_shuffle_epi8(d, r16));                       \
  c = _mm256_add_epi64(c, d);                                                                    \
  b = _mm256_xor_si256(b, c); b = ROT(b, 63, _mm256_or_si256(_mm256_srli_epi64(b, 63), _mm256_add_epi64(b, b)));
#pragma GCC unroll 12
  for (int r = 0; r < 12; r++) {
    const uint8_t* s = SG[r];
    G4(_mm256_setr_epi64x(m[s[0]], m[s[2]], m[s[4]], m[s[6]]), _mm256_setr_epi64x(m[s[1]], m[s[3]], m[s[5]], m[s[7]]));
    b = _mm256_permute4x64_epi64(b, _MM_SHUFFLE(0, 3, 2, 1));
    c = _mm256_permute4x64_epi64(c, _MM_SHUFFLE(1, 0, 3, 2));
    d = _mm256_permute4x64_epi64(d, _MM_SHUFFLE(2, 1, 0, 3));
    G4(_mm256_setr_epi64x(m[s[8]], m[s[10]], m[s[12]], m[s[14]]),
       _mm256_setr_epi64x(m[s[9]], m[s[11]], m[s[13]], m[s[15]]));
    b = _mm256_permute4x64_epi64(b, _MM_SHUFFLE(2, 1, 0, 3));
    c = _mm256_permute4x64_epi64(c, _MM_SHUFFLE(1, 0, 3, 2));
    d = _mm256_permute4x64_epi64(d, _MM_SHUFFLE(0, 3, 2, 1));
  }
  _mm256_storeu_si256((__m256i*)h, _mm256_xor_si256(a0, _mm256_xor_si256(a, c)));
  _mm256_storeu_si256((__m256i*)(h + 4), _mm256_xor_si256(b0, _mm256_xor_si256(b, d)));
}

template <class F>
static double run(F comp, const std::vector<uint8_t>& buf, uint64_t out[8]) {
  uint64_t h[8];
  for (int i = 0; i < 8; i++) h[i] = IV[i];
  h[0] ^= 0x01010000ull ^ 64;
  auto t0 = std::chrono::steady_clock::now();
  const size_t nb = buf.size() / 128;
  for (size_t i = 0; i < nb; i++) comp(h, buf.data() + 128 * i, (uint64_t)(128 * (i + 1)), i + 1 == nb);
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  memcpy(out, h, 64);
  return buf.size() / s / 1e9;
}

int main() {
  std::vector<uint8_t> buf((size_t)512 << 20);
  for (size_t i = 0; i < buf.size(); i++) buf[i] = (uint8_t)(i * 2654435761u >> 11);
  uint64_t ref[8], o[8];
  const bool avx512 = __builtin_cpu_supports("avx512vl");
  for (int rep = 0; rep < 2; rep++) {
    printf("scalar  %.3f GB/s\n", run(comp_scalar, buf, ref));
    if (__builtin_cpu_supports("avx2")) {
      double g = run(comp_vec<false>, buf, o);
      printf("avx2    %.3f GB/s %s\n", g, memcmp(o, ref, 64) ? "MISMATCH" : "ok");
    }
    if (avx512) {
      double g = run(comp_vec<true>, buf, o);
      printf("avx512  %.3f GB/s %s\n", g, memcmp(o, ref, 64) ? "MISMATCH" : "ok");
    }
  }
  return 0;
}
