/*
 * CPU ORACLE (test infrastructure only) — C restatement of the reference's per-point hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library, and
 * only as the checker / CPU baseline. The product path (HIP kernels behind include/kzgpot.h)
 * never links or calls it.
 *
 * Reference being restated (heliaxdev/kzg-setup-powersoftau, Rust; not buildable here — no
 * rustc/cargo, crates not vendored): the algorithms are the pinned third-party crates' own,
 * restated operation by operation so that accept/reject and output bytes match:
 *   - pairing 0.14.2 G1Compressed/G2Compressed::into_affine_unchecked, Fq::sqrt (a^((p-3)/4)),
 *     Fq2::sqrt (Algorithm 9, eprint 2012/685), lexicographic sign rule — called from
 *     powersoftau Accumulator::deserialize at src/bin/preprocess-kgz.rs:105-110.
 *   - src/lib.rs:41-54 read_g1 / :56-80 read_g2 byte reordering, then ark-ec 0.2.0
 *     deserialize_uncompressed: Fp384 x<p, SWFlags, is_in_correct_subgroup_assuming_on_curve =
 *     mul_bits(r).is_zero() with ark's Jacobian double_in_place (a=0) / add_assign_mixed.
 *   - ark serialize_uncompressed (src/bin/preprocess-kgz.rs:188-194, preprocess-fastkgz.rs:193-208).
 *   - the kgz / fastkgz file pipelines (preprocess-kgz.rs:69-199, preprocess-fastkgz.rs:70-213).
 * Arithmetic mirrors ark-ff 0.2 (6 x u64 Montgomery limbs, CIOS with 128-bit products).
 *
 * Parity pinning: see oracle/kzgpot_oracle.py header (spec constants + cross-implementation
 * agreement; reference output digests only when the real transcript is supplied).
 *
 * Build: make -C oracle   (gcc -O2 -fPIC -shared -pthread)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t l[6]; } fp;      /* Montgomery form, fully reduced (< p), like ark-ff */
typedef struct { fp c0, c1; } fp2;

static const uint64_t PM[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                               0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const uint64_t INV = 0x89f3fffcfffcfffdULL; /* -p^{-1} mod 2^64 */
static const uint64_t R2[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL,
                               0x67eb88a9939d83c0ULL, 0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};
static const uint64_t ONE_M[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                                  0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
/* r, big-endian bit iteration (ark BitIteratorBE over Fr::characteristic()) */
static const uint64_t RORD[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                 0x73eda753299d7d48ULL};

/* ----------------------------------------------------------------- Fp (ark-ff 0.2 style) */
static int fp_geq_p(const uint64_t a[6]) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > PM[i]) return 1;
    if (a[i] < PM[i]) return 0;
  }
  return 1;
}
static void sub_p(uint64_t a[6]) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - PM[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);
  }
}
static void fp_add(fp* r, const fp* a, const fp* b) {
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    r->l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (fp_geq_p(r->l)) sub_p(r->l);
}
static void fp_sub(fp* r, const fp* a, const fp* b) {
  uint64_t br = 0;
  uint64_t t[6];
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      u128 s = (u128)t[i] + PM[i] + c;
      t[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  memcpy(r->l, t, sizeof t);
}
static void fp_dbl(fp* r, const fp* a) { fp_add(r, a, a); }
static void fp_neg(fp* r, const fp* a) {
  fp z = {{0}};
  fp_sub(r, &z, a);
}
static void fp_mul(fp* r, const fp* a, const fp* b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 6; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 6; j++) {
      u128 s = (u128)a->l[j] * b->l[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[6] + c;
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * INV;
    s = (u128)m * PM[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < 6; j++) {
      s = (u128)m * PM[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[6] + c;
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  memcpy(r->l, t, 48);
  if (fp_geq_p(r->l)) sub_p(r->l);
}
static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static int fp_is_zero(const fp* a) { return (a->l[0] | a->l[1] | a->l[2] | a->l[3] | a->l[4] | a->l[5]) == 0; }
static int fp_eq(const fp* a, const fp* b) { return memcmp(a->l, b->l, 48) == 0; }
static void fp_one(fp* r) { memcpy(r->l, ONE_M, 48); }
static void fp_zero(fp* r) { memset(r->l, 0, 48); }
/* from_repr: canonical limbs (< p checked by caller) -> Montgomery */
static void fp_from_canon(fp* r, const uint64_t c[6]) {
  fp a, b;
  memcpy(a.l, c, 48);
  memcpy(b.l, R2, 48);
  fp_mul(r, &a, &b);
}
static void fp_to_canon(uint64_t c[6], const fp* a) {
  fp one = {{1, 0, 0, 0, 0, 0}}, t;
  fp_mul(&t, a, &one);
  memcpy(c, t.l, 48);
}
/* exponentiation by a little-endian u64 exponent, MSB-first square-and-multiply (ff `pow`) */
static void fp_pow(fp* r, const fp* a, const uint64_t* e, int nlimbs) {
  fp res;
  fp_one(&res);
  int started = 0;
  for (int i = nlimbs - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      if (started) fp_sqr(&res, &res);
      if ((e[i] >> b) & 1) {
        fp_mul(&res, &res, a);
        started = 1;
      }
    }
  *r = res;
}
static uint64_t E_PM3_4[6], E_PM1_2[6]; /* (p-3)/4, (p-1)/2 */
static fp NEG_ONE;
static pthread_once_t init_once = PTHREAD_ONCE_INIT;
static void init_consts(void) {
  /* (p-3)/4 = p >> 2 (p = 3 mod 4, low bits ...11 → floor division is exact minus 3/4) */
  for (int i = 0; i < 6; i++) E_PM3_4[i] = (PM[i] >> 2) | (i < 5 ? PM[i + 1] << 62 : 0);
  for (int i = 0; i < 6; i++) E_PM1_2[i] = (PM[i] >> 1) | (i < 5 ? PM[i + 1] << 63 : 0);
  fp one;
  fp_one(&one);
  fp_neg(&NEG_ONE, &one);
}
static int cmp_canon(const uint64_t a[6], const uint64_t b[6]) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] < b[i]) return -1;
    if (a[i] > b[i]) return 1;
  }
  return 0;
}
/* pairing Ord for Fq: compare canonical representations */
static int fp_lt(const fp* a, const fp* b) {
  uint64_t ca[6], cb[6];
  fp_to_canon(ca, a);
  fp_to_canon(cb, b);
  return cmp_canon(ca, cb) < 0;
}
/* pairing 0.14.2 Fq::sqrt: a1 = a^((p-3)/4); a0 = a1^2 a; a0 == -1 → None; else a1 a */
static int fq_sqrt(fp* r, const fp* a) {
  fp a1, a0;
  fp_pow(&a1, a, E_PM3_4, 6);
  fp_sqr(&a0, &a1);
  fp_mul(&a0, &a0, a);
  if (fp_eq(&a0, &NEG_ONE)) return 0;
  fp_mul(r, &a1, a);
  return 1;
}

/* ----------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1) */
static void fp2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static void fp2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static void fp2_dbl(fp2* r, const fp2* a) { fp2_add(r, a, a); }
static void fp2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static void fp2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp aa, bb, s0, s1, t;
  fp_mul(&aa, &a->c0, &b->c0);
  fp_mul(&bb, &a->c1, &b->c1);
  fp_add(&s0, &a->c0, &a->c1);
  fp_add(&s1, &b->c0, &b->c1);
  fp_mul(&t, &s0, &s1);
  fp_sub(&t, &t, &aa);
  fp_sub(&r->c1, &t, &bb);
  fp_sub(&r->c0, &aa, &bb);
}
static void fp2_sqr(fp2* r, const fp2* a) { fp2_mul(r, a, a); }
static int fp2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int fp2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void fp2_pow(fp2* r, const fp2* a, const uint64_t* e, int nlimbs) {
  fp2 res;
  fp_one(&res.c0);
  fp_zero(&res.c1);
  int started = 0;
  for (int i = nlimbs - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      if (started) fp2_sqr(&res, &res);
      if ((e[i] >> b) & 1) {
        fp2_mul(&res, &res, a);
        started = 1;
      }
    }
  *r = res;
}
/* pairing 0.14.2 Fq2::sqrt — Algorithm 9 */
static int fq2_sqrt(fp2* r, const fp2* a) {
  if (fp2_is_zero(a)) {
    *r = *a;
    return 1;
  }
  fp2 a1, alpha, a0, t, neg1;
  neg1.c0 = NEG_ONE;
  fp_zero(&neg1.c1);
  fp2_pow(&a1, a, E_PM3_4, 6);
  fp2_sqr(&alpha, &a1);
  fp2_mul(&alpha, &alpha, a);
  a0 = alpha;
  fp_neg(&a0.c1, &a0.c1); /* frobenius_map(1) */
  fp2_mul(&a0, &a0, &alpha);
  if (fp2_eq(&a0, &neg1)) return 0;
  fp2_mul(&a1, &a1, a);
  if (fp2_eq(&alpha, &neg1)) {
    /* a1 * u = (-a1.c1, a1.c0) */
    t.c0 = a1.c1;
    fp_neg(&t.c0, &t.c0);
    t.c1 = a1.c0;
    *r = t;
  } else {
    fp2 one;
    fp_one(&one.c0);
    fp_zero(&one.c1);
    fp2_add(&alpha, &alpha, &one);
    fp2_pow(&alpha, &alpha, E_PM1_2, 6);
    fp2_mul(r, &a1, &alpha);
  }
  return 1;
}
/* pairing Ord for Fq2: lexicographic on (c1, c0) */
static int fp2_lt(const fp2* a, const fp2* b) {
  uint64_t a1[6], b1[6];
  fp_to_canon(a1, &a->c1);
  fp_to_canon(b1, &b->c1);
  int c = cmp_canon(a1, b1);
  if (c) return c < 0;
  return fp_lt(&a->c0, &b->c0);
}

/* ----------------------------------------------------------------- generic Jacobian (ark 0.2) */
#define DEF_CURVE(F, T)                                                                              \
  typedef struct { T x, y, z; } F##_jac;                                                            \
  /* GroupProjective::double_in_place, COEFF_A == 0 (dbl-2009-l) */                                 \
  static void F##_double(F##_jac* p) {                                                               \
    if (F##_is_zero(&p->z)) return;                                                                  \
    T a, b, c, d, e, f, t;                                                                           \
    F##_sqr(&a, &p->x);                                                                              \
    F##_sqr(&b, &p->y);                                                                              \
    F##_sqr(&c, &b);                                                                                 \
    F##_add(&t, &p->x, &b);                                                                          \
    F##_sqr(&t, &t);                                                                                 \
    F##_sub(&t, &t, &a);                                                                             \
    F##_sub(&t, &t, &c);                                                                             \
    F##_dbl(&d, &t);                                                                                 \
    F##_dbl(&e, &a);                                                                                 \
    F##_add(&e, &e, &a);                                                                             \
    F##_sqr(&f, &e);                                                                                 \
    F##_mul(&p->z, &p->z, &p->y);                                                                    \
    F##_dbl(&p->z, &p->z);                                                                           \
    F##_sub(&p->x, &f, &d);                                                                          \
    F##_sub(&p->x, &p->x, &d);                                                                       \
    F##_dbl(&c, &c);                                                                                 \
    F##_dbl(&c, &c);                                                                                 \
    F##_dbl(&c, &c);                                                                                 \
    F##_sub(&t, &d, &p->x);                                                                          \
    F##_mul(&t, &t, &e);                                                                             \
    F##_sub(&p->y, &t, &c);                                                                          \
  }                                                                                                  \
  /* GroupProjective::add_assign_mixed (madd-2007-bl + equal-point branch) */                        \
  static void F##_add_mixed(F##_jac* p, const T* x2, const T* y2, int inf2, const T* one) {          \
    if (inf2) return;                                                                                \
    if (F##_is_zero(&p->z)) {                                                                        \
      p->x = *x2;                                                                                    \
      p->y = *y2;                                                                                    \
      p->z = *one;                                                                                   \
      return;                                                                                        \
    }                                                                                                \
    T z1z1, u2, s2, h, hh, i, j, r, v, t;                                                            \
    F##_sqr(&z1z1, &p->z);                                                                           \
    F##_mul(&u2, x2, &z1z1);                                                                         \
    F##_mul(&s2, y2, &p->z);                                                                         \
    F##_mul(&s2, &s2, &z1z1);                                                                        \
    if (F##_eq(&p->x, &u2) && F##_eq(&p->y, &s2)) {                                                  \
      F##_double(p);                                                                                 \
      return;                                                                                        \
    }                                                                                                \
    F##_sub(&h, &u2, &p->x);                                                                         \
    F##_sqr(&hh, &h);                                                                                \
    F##_dbl(&i, &hh);                                                                                \
    F##_dbl(&i, &i);                                                                                 \
    F##_mul(&j, &h, &i);                                                                             \
    F##_sub(&r, &s2, &p->y);                                                                         \
    F##_dbl(&r, &r);                                                                                 \
    F##_mul(&v, &p->x, &i);                                                                          \
    F##_sqr(&p->x, &r);                                                                              \
    F##_sub(&p->x, &p->x, &j);                                                                       \
    F##_sub(&p->x, &p->x, &v);                                                                       \
    F##_sub(&p->x, &p->x, &v);                                                                       \
    F##_mul(&j, &j, &p->y);                                                                          \
    F##_dbl(&j, &j);                                                                                 \
    F##_sub(&t, &v, &p->x);                                                                          \
    F##_mul(&t, &t, &r);                                                                             \
    F##_sub(&p->y, &t, &j);                                                                          \
    F##_add(&p->z, &p->z, &h);                                                                       \
    F##_sqr(&p->z, &p->z);                                                                           \
    F##_sub(&p->z, &p->z, &z1z1);                                                                    \
    F##_sub(&p->z, &p->z, &hh);                                                                      \
  }                                                                                                  \
  /* GroupAffine::mul_bits(BitIteratorBE(r)).is_zero() */                                            \
  static int F##_in_subgroup_ref(const T* x, const T* y, int inf, const T* zero, const T* one) {     \
    F##_jac acc;                                                                                     \
    acc.x = *zero;                                                                                   \
    acc.y = *one;                                                                                    \
    acc.z = *zero;                                                                                   \
    int started = 0;                                                                                 \
    for (int w = 3; w >= 0; w--)                                                                     \
      for (int b = 63; b >= 0; b--) {                                                                \
        int bit = (RORD[w] >> b) & 1;                                                                \
        if (!started && !bit) continue;                                                              \
        started = 1;                                                                                 \
        F##_double(&acc);                                                                            \
        if (bit) F##_add_mixed(&acc, x, y, inf, one);                                                \
      }                                                                                              \
    return F##_is_zero(&acc.z);                                                                      \
  }

DEF_CURVE(fp, fp)
DEF_CURVE(fp2, fp2)

/* ----------------------------------------------------------------- byte helpers */
static void be48_to_limbs(uint64_t c[6], const uint8_t* b) {
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | b[(5 - i) * 8 + k];
    c[i] = v;
  }
}
static void le48_to_limbs(uint64_t c[6], const uint8_t* b) {
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 7; k >= 0; k--) v = (v << 8) | b[i * 8 + k];
    c[i] = v;
  }
}
static void limbs_to_le48(uint8_t* b, const uint64_t c[6]) {
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[i * 8 + k] = (uint8_t)(c[i] >> (8 * k));
}
static void limbs_to_be48(uint8_t* b, const uint64_t c[6]) {
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[(5 - i) * 8 + (7 - k)] = (uint8_t)(c[i] >> (8 * k));
}
static void fp_to_le48(uint8_t* b, const fp* a) {
  uint64_t c[6];
  fp_to_canon(c, a);
  limbs_to_le48(b, c);
}
static void fp_to_be48(uint8_t* b, const fp* a) {
  uint64_t c[6];
  fp_to_canon(c, a);
  limbs_to_be48(b, c);
}

/* status codes (negated in the API return value) — identical to include/kzgpot.h */
enum { ST_OK = 0, ST_COMPRESSION_MODE = 1, ST_UNEXPECTED_INFO = 2, ST_NOT_IN_FIELD = 3, ST_NOT_ON_CURVE = 4,
       ST_NOT_IN_SUBGROUP = 5, ST_UNEXPECTED_FLAGS = 6, ST_INFINITY = 7 };
#define F_NO_SUBGROUP_CHECK 0x1u

/* ----------------------------------------------------------------- pairing decompress */
typedef struct { fp x, y; int inf; } g1a;
typedef struct { fp2 x, y; int inf; } g2a;

/* G1Compressed::into_affine_unchecked */
static int pairing_g1_decompress(g1a* out, const uint8_t* enc) {
  uint8_t copy[48];
  memcpy(copy, enc, 48);
  if (!(copy[0] & 0x80)) return ST_COMPRESSION_MODE;
  if (copy[0] & 0x40) {
    copy[0] &= 0x3f;
    for (int i = 0; i < 48; i++)
      if (copy[i]) return ST_UNEXPECTED_INFO;
    out->inf = 1;
    return ST_OK;
  }
  int greatest = (copy[0] & 0x20) != 0;
  copy[0] &= 0x1f;
  uint64_t c[6];
  be48_to_limbs(c, copy);
  if (fp_geq_p(c)) return ST_NOT_IN_FIELD;
  fp x, x3b, y, negy, b4;
  fp_from_canon(&x, c);
  uint64_t four[6] = {4, 0, 0, 0, 0, 0};
  fp_from_canon(&b4, four);
  fp_sqr(&x3b, &x);
  fp_mul(&x3b, &x3b, &x);
  fp_add(&x3b, &x3b, &b4);
  if (!fq_sqrt(&y, &x3b)) return ST_NOT_ON_CURVE;
  fp_neg(&negy, &y);
  out->x = x;
  out->y = (fp_lt(&y, &negy) ^ greatest) ? y : negy;
  out->inf = 0;
  return ST_OK;
}
/* G2Compressed::into_affine_unchecked */
static int pairing_g2_decompress(g2a* out, const uint8_t* enc) {
  uint8_t copy[96];
  memcpy(copy, enc, 96);
  if (!(copy[0] & 0x80)) return ST_COMPRESSION_MODE;
  if (copy[0] & 0x40) {
    copy[0] &= 0x3f;
    for (int i = 0; i < 96; i++)
      if (copy[i]) return ST_UNEXPECTED_INFO;
    out->inf = 1;
    return ST_OK;
  }
  int greatest = (copy[0] & 0x20) != 0;
  copy[0] &= 0x1f;
  uint64_t c1[6], c0[6];
  be48_to_limbs(c1, copy);
  be48_to_limbs(c0, copy + 48);
  if (fp_geq_p(c0) || fp_geq_p(c1)) return ST_NOT_IN_FIELD;
  fp2 x, x3b, y, negy, b;
  fp_from_canon(&x.c0, c0);
  fp_from_canon(&x.c1, c1);
  uint64_t four[6] = {4, 0, 0, 0, 0, 0};
  fp_from_canon(&b.c0, four);
  b.c1 = b.c0;
  fp2_sqr(&x3b, &x);
  fp2_mul(&x3b, &x3b, &x);
  fp2_add(&x3b, &x3b, &b);
  if (!fq2_sqrt(&y, &x3b)) return ST_NOT_ON_CURVE;
  fp2_neg(&negy, &y);
  out->x = x;
  out->y = (fp2_lt(&y, &negy) ^ greatest) ? y : negy;
  out->inf = 0;
  return ST_OK;
}
/* G1Uncompressed::from_affine / G2Uncompressed::from_affine */
static void pairing_g1_uncompressed(uint8_t* b, const g1a* p) {
  memset(b, 0, 96);
  if (p->inf) {
    b[0] = 0x40;
    return;
  }
  fp_to_be48(b, &p->x);
  fp_to_be48(b + 48, &p->y);
}
static void pairing_g2_uncompressed(uint8_t* b, const g2a* p) {
  memset(b, 0, 192);
  if (p->inf) {
    b[0] = 0x40;
    return;
  }
  fp_to_be48(b, &p->x.c1);
  fp_to_be48(b + 48, &p->x.c0);
  fp_to_be48(b + 96, &p->y.c1);
  fp_to_be48(b + 144, &p->y.c0);
}

/* ----------------------------------------------------------------- ark side */
/* Fp384 deserialize(_with_flags): returns status; *inf from SWFlags */
static int ark_fp_read(fp* r, const uint8_t* le, int with_flags, int* inf) {
  uint8_t b[48];
  memcpy(b, le, 48);
  if (with_flags) {
    int pos = (b[47] >> 7) & 1, isinf = (b[47] >> 6) & 1;
    if (pos && isinf) return ST_UNEXPECTED_FLAGS;
    *inf = isinf;
    b[47] &= 0x3f;
  }
  uint64_t c[6];
  le48_to_limbs(c, b);
  if (fp_geq_p(c)) return ST_NOT_IN_FIELD;
  fp_from_canon(r, c);
  return ST_OK;
}
/* read_g1 (src/lib.rs:41-54) + deserialize_uncompressed; *a receives the ark point */
static int read_g1(g1a* a, const uint8_t* pairing96, int check) {
  uint8_t ark[96];
  for (int i = 0; i < 48; i++) {
    ark[i] = pairing96[47 - i];
    ark[48 + i] = pairing96[95 - i];
  }
  int inf = 0, st;
  if ((st = ark_fp_read(&a->x, ark, 0, NULL))) return st;
  if ((st = ark_fp_read(&a->y, ark + 48, 1, &inf))) return st;
  a->inf = inf;
  if (check) {
    fp zero, one;
    fp_zero(&zero);
    fp_one(&one);
    if (!fp_in_subgroup_ref(&a->x, &a->y, inf, &zero, &one)) return ST_NOT_IN_SUBGROUP;
  }
  return ST_OK;
}
/* read_g2 (src/lib.rs:56-80) */
static int read_g2(g2a* a, const uint8_t* p, int check) {
  uint8_t ark[192];
  const int src[4] = {48, 0, 144, 96};
  for (int q = 0; q < 4; q++)
    for (int i = 0; i < 48; i++) ark[q * 48 + i] = p[src[q] + 47 - i];
  int inf = 0, st;
  if ((st = ark_fp_read(&a->x.c0, ark, 0, NULL))) return st;
  if ((st = ark_fp_read(&a->x.c1, ark + 48, 0, NULL))) return st;
  if ((st = ark_fp_read(&a->y.c0, ark + 96, 0, NULL))) return st;
  if ((st = ark_fp_read(&a->y.c1, ark + 144, 1, &inf))) return st;
  a->inf = inf;
  if (check) {
    fp2 zero, one;
    fp_zero(&zero.c0);
    fp_zero(&zero.c1);
    fp_one(&one.c0);
    fp_zero(&one.c1);
    if (!fp2_in_subgroup_ref(&a->x, &a->y, inf, &zero, &one)) return ST_NOT_IN_SUBGROUP;
  }
  return ST_OK;
}
/* serialize_uncompressed */
static void ark_g1_serialize(uint8_t* b, const g1a* a) {
  fp_to_le48(b, &a->x);
  fp_to_le48(b + 48, &a->y);
  if (a->inf) b[95] |= 0x40;
}
static void ark_g2_serialize(uint8_t* b, const g2a* a) {
  fp_to_le48(b, &a->x.c0);
  fp_to_le48(b + 48, &a->x.c1);
  fp_to_le48(b + 96, &a->y.c0);
  fp_to_le48(b + 144, &a->y.c1);
  if (a->inf) b[191] |= 0x40;
}
static void ark_g1_zero(g1a* a) { fp_zero(&a->x); fp_one(&a->y); a->inf = 1; }
static void ark_g2_zero(g2a* a) {
  fp_zero(&a->x.c0); fp_zero(&a->x.c1); fp_one(&a->y.c0); fp_zero(&a->y.c1); a->inf = 1;
}

/* ----------------------------------------------------------------- per-point contract */
/* decompression stage (powersoftau decompress_all → into_affine_unchecked) */
static int stage_decompress_g1(g1a* p, const uint8_t* in) { return pairing_g1_decompress(p, in); }
static int stage_decompress_g2(g2a* p, const uint8_t* in) { return pairing_g2_decompress(p, in); }
/* check+emit stage (Accumulator::serialize(No) → read_g1 → serialize_uncompressed) */
static int stage_check_g1(uint8_t* out, const g1a* p, uint32_t flags) {
  g1a a;
  if (flags & F_NO_SUBGROUP_CHECK) {
    if (p->inf) ark_g1_zero(&a); else { a = *p; a.inf = 0; }
    ark_g1_serialize(out, &a);
    return ST_OK;
  }
  uint8_t un[96];
  pairing_g1_uncompressed(un, p);
  int st = read_g1(&a, un, 1);
  if (st) return p->inf ? ST_INFINITY : st;
  ark_g1_serialize(out, &a);
  return ST_OK;
}
static int stage_check_g2(uint8_t* out, const g2a* p, uint32_t flags) {
  g2a a;
  if (flags & F_NO_SUBGROUP_CHECK) {
    if (p->inf) ark_g2_zero(&a); else { a = *p; a.inf = 0; }
    ark_g2_serialize(out, &a);
    return ST_OK;
  }
  uint8_t un[192];
  pairing_g2_uncompressed(un, p);
  int st = read_g2(&a, un, 1);
  if (st) return p->inf ? ST_INFINITY : st;
  ark_g2_serialize(out, &a);
  return ST_OK;
}

/* ----------------------------------------------------------------- threading */
typedef struct {
  int kind; /* 0 g1 decompress, 1 g2 decompress, 2 g1 check, 3 g2 check, 4 g1 transcode, 5 g2 transcode */
  const uint8_t* in;
  uint8_t* out;
  void* pts;
  uint8_t* st;
  size_t lo, hi;
  uint32_t flags;
} job_t;

static void* run_job(void* arg) {
  job_t* j = (job_t*)arg;
  for (size_t i = j->lo; i < j->hi; i++) {
    int s = ST_OK;
    switch (j->kind) {
      case 0: s = stage_decompress_g1(&((g1a*)j->pts)[i], j->in + 48 * i); break;
      case 1: s = stage_decompress_g2(&((g2a*)j->pts)[i], j->in + 96 * i); break;
      case 2: if (j->st[i] == ST_OK) s = stage_check_g1(j->out + 96 * i, &((g1a*)j->pts)[i], j->flags); else s = j->st[i]; break;
      case 3: if (j->st[i] == ST_OK) s = stage_check_g2(j->out + 192 * i, &((g2a*)j->pts)[i], j->flags); else s = j->st[i]; break;
      case 4: {
        g1a a;
        s = read_g1(&a, j->in + 96 * i, 1);
        if (!s) ark_g1_serialize(j->out + 96 * i, &a);
        break;
      }
      case 5: {
        g2a a;
        s = read_g2(&a, j->in + 192 * i, 1);
        if (!s) ark_g2_serialize(j->out + 192 * i, &a);
        break;
      }
    }
    j->st[i] = (uint8_t)s;
  }
  return NULL;
}

/* contiguous chunks of len/threads (powersoftau decompress_all's schedule) */
static void run_parallel(int kind, const uint8_t* in, uint8_t* out, void* pts, uint8_t* st, size_t n,
                         uint32_t flags, int threads) {
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  pthread_t tid[256];
  job_t jobs[256];
  if (threads > 256) threads = 256;
  size_t chunk = n / threads + (n % threads != 0);
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){kind, in, out, pts, st, t * chunk, (t + 1) * chunk < n ? (t + 1) * chunk : n, flags};
    if (jobs[t].lo > n) jobs[t].lo = n;
    if (threads == 1)
      run_job(&jobs[t]);
    else
      pthread_create(&tid[t], NULL, run_job, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

static int finish(uint8_t* st, size_t n, uint8_t* out, size_t out_rec, int64_t* first_bad, uint8_t* status) {
  int ret = 0;
  int64_t fb = -1;
  for (size_t i = 0; i < n; i++) {
    if (st[i] != ST_OK) {
      memset(out + out_rec * i, 0, out_rec);
      if (fb < 0) {
        fb = (int64_t)i;
        ret = -(int)st[i];
      }
    }
  }
  if (first_bad) *first_bad = fb;
  if (status) memcpy(status, st, n);
  return ret;
}

/* ----------------------------------------------------------------- exported oracle API */
/* a failed allocation: the library's KZGPOT_E_OUT_OF_MEMORY (include/kzgpot.h) */
#define ORACLE_E_NOMEM (-108)
/* threads_decompress: workers for the decompression stage (reference: num_cpus);
 * threads_check: workers for the read_g1/read_g2 + serialize stage (reference: 1). */
int oracle_g1_decompress(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad,
                         uint8_t* status, int threads_decompress, int threads_check) {
  pthread_once(&init_once, init_consts);
  g1a* pts = (g1a*)calloc(n ? n : 1, sizeof(g1a));
  uint8_t* st = (uint8_t*)calloc(n ? n : 1, 1);
  if (!pts || !st) return free(pts), free(st), ORACLE_E_NOMEM;
  run_parallel(0, in, out, pts, st, n, flags, threads_decompress);
  run_parallel(2, in, out, pts, st, n, flags, threads_check);
  int r = finish(st, n, out, 96, first_bad, status);
  free(pts);
  free(st);
  return r;
}
int oracle_g2_decompress(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad,
                         uint8_t* status, int threads_decompress, int threads_check) {
  pthread_once(&init_once, init_consts);
  g2a* pts = (g2a*)calloc(n ? n : 1, sizeof(g2a));
  uint8_t* st = (uint8_t*)calloc(n ? n : 1, 1);
  if (!pts || !st) return free(pts), free(st), ORACLE_E_NOMEM;
  run_parallel(1, in, out, pts, st, n, flags, threads_decompress);
  run_parallel(3, in, out, pts, st, n, flags, threads_check);
  int r = finish(st, n, out, 192, first_bad, status);
  free(pts);
  free(st);
  return r;
}
int oracle_g1_transcode(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad, uint8_t* status, int threads) {
  pthread_once(&init_once, init_consts);
  uint8_t* st = (uint8_t*)calloc(n ? n : 1, 1);
  if (!st) return ORACLE_E_NOMEM;
  run_parallel(4, in, out, NULL, st, n, 0, threads);
  int r = finish(st, n, out, 96, first_bad, status);
  free(st);
  return r;
}
int oracle_g2_transcode(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad, uint8_t* status, int threads) {
  pthread_once(&init_once, init_consts);
  uint8_t* st = (uint8_t*)calloc(n ? n : 1, 1);
  if (!st) return ORACLE_E_NOMEM;
  run_parallel(5, in, out, NULL, st, n, 0, threads);
  int r = finish(st, n, out, 192, first_bad, status);
  free(st);
  return r;
}

/* powersoftau CONTRIBUTION_BYTE_SIZE for N powers */
size_t oracle_contribution_size(uint64_t n) {
  return (2 * n - 1) * 48 + n * 96 + 2 * n * 48 + 96 + (3 * 192 + 6 * 96) + 64;
}
size_t oracle_output_size(uint64_t n, int fast) {
  return fast ? (2 * n - 1) * 96 + n * 96 + 2 * 192 + n * 192 : (2 * n - 1) * 96 + n * 96 + 576;
}

/* preprocess-kgz.rs / preprocess-fastkgz.rs main on an in-memory transcript.
 * Returns 0, or -(status) of the first failing point in reference section order; *bad_section /
 * *bad_index locate it. */
int oracle_preprocess(const uint8_t* tr, size_t len, uint64_t n, int fast, uint8_t* out, int threads,
                      int* bad_section, int64_t* bad_index) {
  pthread_once(&init_once, init_consts);
  if (len != oracle_contribution_size(n)) return -103;
  const uint8_t* p = tr + 64;
  const size_t cnt[5] = {2 * n - 1, n, n, n, 1};
  const int isg2[5] = {0, 1, 0, 0, 1};
  const int checked[5] = {1, 1, 1, fast ? 1 : 0, 0};
  uint8_t* outs[5];
  int64_t fb;
  int ret = 0;
  for (int s = 0; s < 5; s++) {
    size_t rec_in = isg2[s] ? 96 : 48, rec_out = isg2[s] ? 192 : 96;
    outs[s] = (uint8_t*)malloc(cnt[s] * rec_out);
    if (!outs[s]) {
      for (int k = 0; k < s; k++) free(outs[k]);
      return ORACLE_E_NOMEM;
    }
    uint32_t fl = checked[s] ? 0 : F_NO_SUBGROUP_CHECK;
    int r = isg2[s] ? oracle_g2_decompress(p, cnt[s], outs[s], fl, &fb, NULL, threads, threads)
                    : oracle_g1_decompress(p, cnt[s], outs[s], fl, &fb, NULL, threads, threads);
    if (r && !ret) {
      ret = r;
      if (bad_section) *bad_section = s;
      if (bad_index) *bad_index = fb;
    }
    p += cnt[s] * rec_in;
  }
  if (!ret) {
    uint8_t* o = out;
    memcpy(o, outs[0], cnt[0] * 96); o += cnt[0] * 96;
    memcpy(o, outs[2], cnt[2] * 96); o += cnt[2] * 96;
    if (!fast) {
      memcpy(o, outs[0], 96); o += 96;               /* g = τG1[0] */
      memcpy(o, outs[2], 96); o += 96;               /* gamma_g = ατG1[0] */
      memcpy(o, outs[1], 192); o += 192;             /* h = τG2[0] */
      memcpy(o, outs[1] + 192, 192); o += 192;       /* beta_h = τG2[1] */
    } else {
      memcpy(o, outs[1], 192); o += 192;             /* h */
      memcpy(o, outs[1] + 192, 192); o += 192;       /* beta_h */
      memcpy(o, outs[1], cnt[1] * 192); o += cnt[1] * 192; /* powers_of_h */
    }
  }
  for (int s = 0; s < 5; s++) free(outs[s]);
  return ret;
}

/* ----------------------------------------------------------------- synthetic data helpers */
/* [k]G for a big-endian 32-byte scalar k (tests only; same Jacobian formulas) */
static const uint64_t G1X[6] = {0xfb3af00adb22c6bbULL, 0x6c55e83ff97a1aefULL, 0xa14e3a3f171bac58ULL,
                                0xc3688c4f9774b905ULL, 0x2695638c4fa9ac0fULL, 0x17f1d3a73197d794ULL};
static const uint64_t G1Y[6] = {0x0caa232946c5e7e1ULL, 0xd03cc744a2888ae4ULL, 0x00db18cb2c04b3edULL,
                                0xfcf5e095d5d00af6ULL, 0xa09e30ed741d8ae4ULL, 0x08b3f481e3aaa0f1ULL};
static void fp_inv(fp* r, const fp* a) {
  uint64_t e[6];
  memcpy(e, PM, 48);
  e[0] -= 2;
  fp_pow(r, a, e, 6);
}
/* writes pairing-compressed (48 B) and ark-uncompressed (96 B) encodings of [k_i]G1 */
int oracle_g1_scalar_mul_encode(const uint8_t* scalars_be32, size_t n, uint8_t* compressed, uint8_t* ark) {
  pthread_once(&init_once, init_consts);
  fp gx, gy, zero, one;
  fp_from_canon(&gx, G1X);
  fp_from_canon(&gy, G1Y);
  fp_zero(&zero);
  fp_one(&one);
  for (size_t i = 0; i < n; i++) {
    fp_jac acc = {zero, one, zero};
    const uint8_t* k = scalars_be32 + 32 * i;
    int started = 0;
    for (int byte = 0; byte < 32; byte++)
      for (int b = 7; b >= 0; b--) {
        int bit = (k[byte] >> b) & 1;
        if (!started && !bit) continue;
        started = 1;
        fp_double(&acc);
        if (bit) fp_add_mixed(&acc, &gx, &gy, 0, &one);
      }
    uint8_t* c = compressed + 48 * i;
    uint8_t* a = ark + 96 * i;
    if (fp_is_zero(&acc.z)) {
      memset(c, 0, 48);
      c[0] = 0xc0;
      memset(a, 0, 96);
      a[48] = 1; /* ark zero() = (0, 1, inf) */
      a[95] |= 0x40;
      continue;
    }
    fp zi, zi2, x, y, ny;
    fp_inv(&zi, &acc.z);
    fp_sqr(&zi2, &zi);
    fp_mul(&x, &acc.x, &zi2);
    fp_mul(&y, &acc.y, &zi2);
    fp_mul(&y, &y, &zi);
    fp_neg(&ny, &y);
    fp_to_be48(c, &x);
    c[0] |= 0x80;
    if (fp_lt(&ny, &y)) c[0] |= 0x20;
    fp_to_le48(a, &x);
    fp_to_le48(a + 48, &y);
  }
  return 0;
}

/* ----------------------------------------------------------------- the reference pipeline, file to file */
/* preprocess-kgz.rs / preprocess-fastkgz.rs `main` in the reference's own shape, for the CPU
 * baseline beside the GPU end-to-end rows (bench.py cpu_baseline.e2e). Stage by stage:
 *   0 download_parameters (preprocess-kgz.rs:32-67): read the whole transcript, BLAKE2b-512, compare;
 *   1 powersoftau_uncompress (:69-111): a HashReader (BLAKE2b of every byte read) over an 8 KiB
 *     BufReader; Accumulator::deserialize(Yes, No) reads each section's encodings one record at a
 *     time, then decompress_all (powersoftau lib.rs) splits the section into chunks of
 *     len / num_cpus points (at least 1) and runs into_affine_unchecked on one thread per chunk;
 *   2 Accumulator::serialize(No) (:112-125): every point's pairing-uncompressed encoding through an
 *     8 KiB BufWriter into a new `powersoftau_uncompressed` file (create_new);
 *   3 load_powersoftau_accumulator (:128-160, fastkgz :129-178): a 1 MiB BufReader, read_g1 / read_g2
 *     (src/lib.rs:41-80: ark deserialize_uncompressed, subgroup check mul_bits(r)) on one thread —
 *     τG1, τG2, ατG1 (+ βτG1 for fastkgz);
 *   4 the output (:186-194, fastkgz :190-208): File::create, then serialize_uncompressed per point
 *     straight to the unbuffered File: one write() per Fp coordinate (2 per G1 point, 4 per G2).
 * stage_s[0..4] receive the stage times. Returns 0, -(status) of a rejected point, -102 (I/O),
 * -103 (size) or -104 (digest mismatch, when expect_hex is given). digest_hex (129 B, may be NULL)
 * receives the transcript's BLAKE2b. */
#include <fcntl.h>
#include <stdio.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "blake2b_ref.h"

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int write_all_fd(int fd, const uint8_t* p, size_t n) {
  while (n) {
    ssize_t w = write(fd, p, n);
    if (w <= 0) return -1;
    p += w, n -= (size_t)w;
  }
  return 0;
}

/* std::io::BufReader: a read at least as large as the buffer bypasses it when it is empty */
typedef struct { int fd; uint8_t* buf; size_t cap, pos, len; oracle_blake2b_state* hash; } breader;
static int br_read_exact(breader* r, uint8_t* dst, size_t n) {
  uint8_t* d0 = dst;
  size_t n0 = n;
  while (n) {
    if (r->pos == r->len) {
      if (n >= r->cap) {
        ssize_t k = read(r->fd, dst, n);
        if (k <= 0) return -1;
        dst += k, n -= (size_t)k;
        continue;
      }
      ssize_t k = read(r->fd, r->buf, r->cap);
      if (k <= 0) return -1;
      r->pos = 0, r->len = (size_t)k;
    }
    size_t m = r->len - r->pos < n ? r->len - r->pos : n;
    memcpy(dst, r->buf + r->pos, m);
    r->pos += m, dst += m, n -= m;
  }
  if (r->hash) oracle_blake2b_update(r->hash, d0, n0); /* HashReader: every byte handed out */
  return 0;
}

/* std::io::BufWriter */
typedef struct { int fd; uint8_t* buf; size_t cap, len; int err; } bwriter;
static void bw_flush(bwriter* w) {
  if (w->len && write_all_fd(w->fd, w->buf, w->len)) w->err = 1;
  w->len = 0;
}
static void bw_write_all(bwriter* w, const uint8_t* p, size_t n) {
  if (w->len + n > w->cap) bw_flush(w);
  if (n >= w->cap) {
    if (write_all_fd(w->fd, p, n)) w->err = 1;
    return;
  }
  memcpy(w->buf + w->len, p, n);
  w->len += n;
}

typedef struct {
  int g2;
  const uint8_t* enc;
  void* pts;
  size_t lo, hi;
  int64_t bad;
  int st;
} dchunk;
static void* decompress_chunk(void* arg) {
  dchunk* c = (dchunk*)arg;
  for (size_t i = c->lo; i < c->hi; i++) {
    int s = c->g2 ? pairing_g2_decompress(&((g2a*)c->pts)[i], c->enc + 96 * i)
                  : pairing_g1_decompress(&((g1a*)c->pts)[i], c->enc + 48 * i);
    if (s && c->bad < 0) c->bad = (int64_t)i, c->st = s;
  }
  return NULL;
}
/* powersoftau decompress_all: chunk_size = len / num_cpus (min 1), one scoped thread per chunk */
static int decompress_all(int g2, const uint8_t* enc, void* pts, size_t len, int num_cpus) {
  size_t chunk = len / (size_t)(num_cpus > 0 ? num_cpus : 1);
  if (chunk == 0) chunk = 1;
  size_t nt = (len + chunk - 1) / chunk;
  dchunk* cs = (dchunk*)calloc(nt ? nt : 1, sizeof(dchunk));
  pthread_t* tid = (pthread_t*)calloc(nt ? nt : 1, sizeof(pthread_t));
  if (!cs || !tid) return free(cs), free(tid), -ORACLE_E_NOMEM; /* the caller negates */
  for (size_t t = 0; t < nt; t++) {
    cs[t] = (dchunk){g2, enc, pts, t * chunk, (t + 1) * chunk < len ? (t + 1) * chunk : len, -1, 0};
    if (pthread_create(&tid[t], NULL, decompress_chunk, &cs[t])) decompress_chunk(&cs[t]), tid[t] = 0;
  }
  int st = 0;
  for (size_t t = 0; t < nt; t++) {
    if (tid[t]) pthread_join(tid[t], NULL);
    if (!st && cs[t].bad >= 0) st = cs[t].st; /* the reference keeps an arbitrary one; we keep the first */
  }
  free(cs);
  free(tid);
  return st;
}

int oracle_preprocess_pipeline(const char* transcript_path, const char* uncompressed_path, const char* out_path,
                               uint64_t n, int fast, int num_cpus, const char* expect_hex, char* digest_hex,
                               double* stage_s) {
  pthread_once(&init_once, init_consts);
  double t0 = now_s(), st_s[5] = {0, 0, 0, 0, 0};
  const size_t len = oracle_contribution_size(n);
  int ret = 0;
  /* 0: download_parameters' check_file_hash on the existing file (read_to_end + BLAKE2b) */
  {
    int fd = open(transcript_path, O_RDONLY);
    if (fd < 0) return -102;
    struct stat sb;
    if (fstat(fd, &sb) || (size_t)sb.st_size != len) {
      close(fd);
      return -103;
    }
    uint8_t* all = (uint8_t*)malloc(len);
    if (!all) {
      close(fd);
      return ORACLE_E_NOMEM;
    }
    size_t got = 0;
    while (got < len) {
      ssize_t k = read(fd, all + got, len - got);
      if (k <= 0) break;
      got += (size_t)k;
    }
    close(fd);
    uint8_t d[64];
    oracle_blake2b(all, got, d);
    free(all);
    char hex[129];
    for (int i = 0; i < 64; i++) snprintf(hex + 2 * i, 3, "%02x", d[i]);
    if (digest_hex) memcpy(digest_hex, hex, 129);
    if (got != len) return -102;
    if (expect_hex && strncmp(hex, expect_hex, 128) != 0) return -104;
  }
  st_s[0] = now_s() - t0;
  const size_t cnt[5] = {2 * n - 1, n, n, n, 1};
  const int isg2[5] = {0, 1, 0, 0, 1};
  void* pts[5] = {0, 0, 0, 0, 0};
  /* 1: Accumulator::deserialize(UseCompression::Yes, CheckForCorrectness::No) behind HashReader */
  t0 = now_s();
  {
    int fd = open(transcript_path, O_RDONLY);
    if (fd < 0) return -102;
    oracle_blake2b_state h;
    oracle_blake2b_init(&h);
    breader r = {fd, (uint8_t*)malloc(8192), 8192, 0, 0, &h};
    uint8_t hash64[64];
    if (!r.buf) ret = ORACLE_E_NOMEM;
    else if (br_read_exact(&r, hash64, 64)) ret = -102;
    for (int s = 0; s < 5 && !ret; s++) {
      const size_t rec = isg2[s] ? 96 : 48;
      uint8_t* enc = (uint8_t*)malloc(cnt[s] * rec);
      pts[s] = calloc(cnt[s], isg2[s] ? sizeof(g2a) : sizeof(g1a));
      if (!enc || !pts[s]) ret = ORACLE_E_NOMEM;
      for (size_t i = 0; i < cnt[s] && !ret; i++)
        if (br_read_exact(&r, enc + rec * i, rec)) ret = -102;
      if (!ret) {
        int e = decompress_all(isg2[s], enc, pts[s], cnt[s], num_cpus);
        if (e) ret = -e;
      }
      free(enc);
    }
    free(r.buf);
    close(fd);
  }
  st_s[1] = now_s() - t0;
  /* 2: Accumulator::serialize(UseCompression::No) through an 8 KiB BufWriter */
  t0 = now_s();
  if (!ret) {
    int fd = open(uncompressed_path, O_WRONLY | O_CREAT | O_EXCL, 0644);
    if (fd < 0) ret = -102;
    else {
      bwriter w = {fd, (uint8_t*)malloc(8192), 8192, 0, 0};
      uint8_t b[192];
      if (!w.buf) ret = ORACLE_E_NOMEM, w.err = 1;
      for (int s = 0; s < 5 && w.buf; s++)
        for (size_t i = 0; i < cnt[s]; i++) {
          if (isg2[s]) pairing_g2_uncompressed(b, &((g2a*)pts[s])[i]);
          else pairing_g1_uncompressed(b, &((g1a*)pts[s])[i]);
          bw_write_all(&w, b, isg2[s] ? 192 : 96);
        }
      if (w.buf) bw_flush(&w);
      if (w.err && !ret) ret = -102;
      free(w.buf);
      if (close(fd)) ret = -102;
    }
  }
  for (int s = 0; s < 5; s++) free(pts[s]);
  st_s[2] = now_s() - t0;
  /* 3: load_powersoftau_accumulator: read_g1 / read_g2 on one thread through a 1 MiB BufReader */
  t0 = now_s();
  const int nload = fast ? 4 : 3; /* τG1, τG2, ατG1 (+ βτG1) */
  void* ark[4] = {0, 0, 0, 0};
  if (!ret) {
    int fd = open(uncompressed_path, O_RDONLY);
    if (fd < 0) ret = -102;
    else {
      breader r = {fd, (uint8_t*)malloc(1 << 20), 1 << 20, 0, 0, NULL};
      uint8_t b[192];
      if (!r.buf) ret = ORACLE_E_NOMEM;
      for (int s = 0; s < nload && !ret; s++) {
        ark[s] = calloc(cnt[s], isg2[s] ? sizeof(g2a) : sizeof(g1a));
        if (!ark[s]) {
          ret = ORACLE_E_NOMEM;
          break;
        }
        for (size_t i = 0; i < cnt[s] && !ret; i++) {
          if (br_read_exact(&r, b, isg2[s] ? 192 : 96)) {
            ret = -102;
            break;
          }
          int e = isg2[s] ? read_g2(&((g2a*)ark[s])[i], b, 1) : read_g1(&((g1a*)ark[s])[i], b, 1);
          if (e) ret = -e; /* read_g1(f).unwrap() */
        }
      }
      free(r.buf);
      close(fd);
    }
  }
  st_s[3] = now_s() - t0;
  /* 4: serialize_uncompressed per point to the unbuffered File */
  t0 = now_s();
  if (!ret) {
    int fd = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) ret = -102;
    else {
      uint8_t b[192];
      int err = 0;
#define W1(P)                                                               \
  do {                                                                      \
    ark_g1_serialize(b, (P));                                               \
    err |= write_all_fd(fd, b, 48) | write_all_fd(fd, b + 48, 48);          \
  } while (0)
#define W2(P)                                                               \
  do {                                                                      \
    ark_g2_serialize(b, (P));                                               \
    for (int q = 0; q < 4; q++) err |= write_all_fd(fd, b + 48 * q, 48);    \
  } while (0)
      g1a* tg1 = (g1a*)ark[0];
      g2a* tg2 = (g2a*)ark[1];
      g1a* ag1 = (g1a*)ark[2];
      for (size_t i = 0; i < cnt[0]; i++) W1(&tg1[i]); /* powers_of_g */
      for (size_t i = 0; i < cnt[2]; i++) W1(&ag1[i]); /* powers_of_gamma_g */
      if (!fast) {                                    /* VerifierKey {g, gamma_g, h, beta_h} */
        W1(&tg1[0]);
        W1(&ag1[0]);
        W2(&tg2[0]);
        W2(&tg2[1]);
      } else { /* h, beta_h, neg_powers_of_h (empty), powers_of_h */
        W2(&tg2[0]);
        W2(&tg2[1]);
        for (size_t i = 0; i < cnt[1]; i++) W2(&tg2[i]);
      }
#undef W1
#undef W2
      if (close(fd) || err) ret = -102;
    }
  }
  for (int s = 0; s < 4; s++) free(ark[s]);
  st_s[4] = now_s() - t0;
  if (stage_s) memcpy(stage_s, st_s, sizeof st_s);
  return ret;
}
