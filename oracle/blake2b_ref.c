/*
 * CPU ORACLE (test infrastructure only) — BLAKE2b-512 for the reference-pipeline restatement.
 *
 * The reference hashes its transcript twice: download_parameters' check_file_hash with
 * blake2b_simd 0.5.11 (src/bin/preprocess-kgz.rs:36-39) and powersoftau's HashReader (the
 * `blake2` 0.6 crate) around the deserializing reader (preprocess-kgz.rs:94-95). Both compute
 * unkeyed BLAKE2b-512 as published in RFC 7693; this is a plain restatement of that RFC (section
 * 3.2 compression, 2.7 message schedule) so that oracle/kzgpot_ref.c's pipeline can time those
 * passes without linking the product's csrc/blake2b.cpp. Only bench.py's cpu_baseline leg and
 * tests/ use it; tests/test_oracle.py checks it against hashlib.blake2b.
 */
#include <stdint.h>
#include <string.h>

#include "blake2b_ref.h"

static const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                               0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                               0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

static const uint8_t SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static uint64_t rotr(uint64_t x, int k) { return (x >> k) | (x << (64 - k)); }

static uint64_t load64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

/* RFC 7693 §3.2 F: compress one 128-byte block; last = final-block flag */
static void compress(oracle_blake2b_state* s, const uint8_t* block, int last) {
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; i++) m[i] = load64(block + 8 * i);
  for (int i = 0; i < 8; i++) v[i] = s->h[i], v[i + 8] = IV[i];
  v[12] ^= s->t[0];
  v[13] ^= s->t[1];
  if (last) v[14] = ~v[14];
#define G(a, b, c, d, x, y)        \
  do {                             \
    v[a] = v[a] + v[b] + (x);      \
    v[d] = rotr(v[d] ^ v[a], 32);  \
    v[c] = v[c] + v[d];            \
    v[b] = rotr(v[b] ^ v[c], 24);  \
    v[a] = v[a] + v[b] + (y);      \
    v[d] = rotr(v[d] ^ v[a], 16);  \
    v[c] = v[c] + v[d];            \
    v[b] = rotr(v[b] ^ v[c], 63);  \
  } while (0)
  for (int r = 0; r < 12; r++) {
    const uint8_t* z = SIGMA[r];
    G(0, 4, 8, 12, m[z[0]], m[z[1]]);
    G(1, 5, 9, 13, m[z[2]], m[z[3]]);
    G(2, 6, 10, 14, m[z[4]], m[z[5]]);
    G(3, 7, 11, 15, m[z[6]], m[z[7]]);
    G(0, 5, 10, 15, m[z[8]], m[z[9]]);
    G(1, 6, 11, 12, m[z[10]], m[z[11]]);
    G(2, 7, 8, 13, m[z[12]], m[z[13]]);
    G(3, 4, 9, 14, m[z[14]], m[z[15]]);
  }
#undef G
  for (int i = 0; i < 8; i++) s->h[i] ^= v[i] ^ v[i + 8];
}

void oracle_blake2b_init(oracle_blake2b_state* s) {
  memcpy(s->h, IV, sizeof IV);
  s->h[0] ^= 0x01010000ULL ^ 64; /* parameter block: digest length 64, no key, fanout = depth = 1 */
  s->t[0] = s->t[1] = 0;
  s->fill = 0;
}

void oracle_blake2b_update(oracle_blake2b_state* s, const uint8_t* p, size_t n) {
  while (n) {
    /* a full buffer is compressed only once more input follows: the last block gets the flag */
    if (s->fill == 128) {
      s->t[0] += 128;
      if (s->t[0] < 128) s->t[1]++;
      compress(s, s->buf, 0);
      s->fill = 0;
    }
    size_t k = 128 - s->fill;
    if (k > n) k = n;
    memcpy(s->buf + s->fill, p, k);
    s->fill += k;
    p += k;
    n -= k;
  }
}

void oracle_blake2b_final(oracle_blake2b_state* s, uint8_t out[64]) {
  s->t[0] += s->fill;
  if (s->t[0] < s->fill) s->t[1]++;
  memset(s->buf + s->fill, 0, 128 - s->fill);
  compress(s, s->buf, 1);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(s->h[i] >> (8 * j));
}

int oracle_blake2b(const uint8_t* p, size_t n, uint8_t out[64]) {
  oracle_blake2b_state s;
  oracle_blake2b_init(&s);
  oracle_blake2b_update(&s, p, n);
  oracle_blake2b_final(&s, out);
  return 0;
}
