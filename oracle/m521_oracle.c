/*
 * m521_oracle.c — CPU restatement of delta-node's Shamir hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Imported solely by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg, always as the checker, never as the thing
 * measured or shipped.  Parity of this restatement is pinned by the golden
 * fixtures in tests/golden/ (generated from the real reference, see
 * tests/golden/make_golden.py) — tests/test_oracle.py checks it against them.
 *
 * Deliberately independent of the product's arithmetic: 9 x 64-bit limbs with
 * unsigned __int128 products (the device uses 17 x 32-bit limbs), a literal
 * `% p` after every Horner step, and the reference's nums/dens/den sequence of
 * field divisions for reconstruct.
 *
 *   PRIME                          delta_node/crypto/shamir/shamir.py:16
 *   _eval_at (Horner, % p)         shamir.py:19-25
 *   make_shares coefficient draw   shamir.py:59-61 -> random.randint(1, p-1)
 *   resolve_shares                 shamir.py:68-90 (nums/dens :77-83, sum :86-89, /den :90)
 *   inverse_mod / div_mod          op.py:16-29 (here by Fermat: a^(p-2), same value)
 *   MT19937 + init_by_array        CPython Modules/_randommodule.c (random.seed(int))
 */
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;
#define NL 9 /* 9 x 64 = 576 bits */

typedef struct { uint64_t w[NL]; } fe; /* canonical residue < p */

/* ----------------------------------------------------------- field ops */
static int fe_is_p_or_more(const fe* a) {
  /* a < 2^522 assumed; a >= p  <=>  bit 521 set or a == p */
  if (a->w[8] >> 9) return 1;
  if (a->w[8] != 0x1FF) return 0;
  for (int i = 0; i < 8; ++i)
    if (a->w[i] != ~0ull) return 0;
  return 1;
}

static void fe_sub_p(fe* a) { /* a -= p  ==  a - 2^521 + 1 */
  a->w[8] -= (1ull << 9);
  for (int i = 0; i < NL; ++i) {
    if (++a->w[i] != 0) break;
  }
}

/* reduce a 1088-bit value (17 x 64 limbs) mod p */
static fe fe_reduce_wide(const uint64_t* x, int nlimbs) {
  uint64_t t[18];
  memset(t, 0, sizeof(t));
  memcpy(t, x, (size_t)nlimbs * 8);
  for (;;) {
    /* hi = t >> 521 ; lo = t mod 2^521 */
    uint64_t hi[18];
    int any = 0;
    for (int i = 0; i < 18; ++i) {
      const int b = 521 + 64 * i;
      const int li = b / 64, sh = b % 64;
      uint64_t v = 0;
      if (li < 18) v = t[li] >> sh;
      if (li + 1 < 18 && sh) v |= t[li + 1] << (64 - sh);
      hi[i] = v;
      any |= (v != 0);
    }
    if (!any) break;
    t[8] &= 0x1FF;
    for (int i = 9; i < 18; ++i) t[i] = 0;
    u128 c = 0;
    for (int i = 0; i < 18; ++i) {
      c += (u128)t[i] + hi[i];
      t[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  fe r;
  memcpy(r.w, t, sizeof(r.w));
  while (fe_is_p_or_more(&r)) fe_sub_p(&r);
  return r;
}

static fe fe_mul(const fe* a, const fe* b) {
  uint64_t p[18];
  memset(p, 0, sizeof(p));
  for (int i = 0; i < NL; ++i) {
    u128 c = 0;
    for (int j = 0; j < NL; ++j) {
      c += (u128)a->w[i] * b->w[j] + p[i + j];
      p[i + j] = (uint64_t)c;
      c >>= 64;
    }
    p[i + NL] = (uint64_t)c;
  }
  return fe_reduce_wide(p, 18);
}

static fe fe_add(const fe* a, const fe* b) {
  uint64_t t[NL];
  u128 c = 0;
  for (int i = 0; i < NL; ++i) {
    c += (u128)a->w[i] + b->w[i];
    t[i] = (uint64_t)c;
    c >>= 64;
  }
  return fe_reduce_wide(t, NL);
}

static fe fe_from_u64(uint64_t v) {
  fe r;
  memset(&r, 0, sizeof(r));
  r.w[0] = v;
  return r;
}

static fe fe_neg(const fe* a) { /* p - a */
  fe r;
  int zero = 1;
  for (int i = 0; i < NL; ++i) zero &= (a->w[i] == 0);
  if (zero) return *a;
  for (int i = 0; i < 8; ++i) r.w[i] = ~a->w[i];
  r.w[8] = (~a->w[8]) & 0x1FF;
  return r;
}

/* signed small integer (|v| < 2^127) -> field element */
static fe fe_from_i128(__int128 v) {
  const int neg = v < 0;
  u128 m = neg ? (u128)(-v) : (u128)v;
  fe r;
  memset(&r, 0, sizeof(r));
  r.w[0] = (uint64_t)m;
  r.w[1] = (uint64_t)(m >> 64);
  return neg ? fe_neg(&r) : r;
}

static fe fe_inv(const fe* a) { /* a^(p-2) : the value op.inverse_mod returns */
  fe r = fe_from_u64(1), b = *a;
  for (int bit = 0; bit < 521; ++bit) {
    if (bit != 1) r = fe_mul(&r, &b); /* p-2 = 2^521-3: bit 1 is the only clear bit */
    b = fe_mul(&b, &b);
  }
  return r;
}

/* limbs: 17 x u32 little endian <-> fe */
static fe fe_load32(const uint32_t* l) {
  fe r;
  memset(&r, 0, sizeof(r));
  for (int i = 0; i < 17; ++i) r.w[i / 2] |= (uint64_t)l[i] << (32 * (i % 2));
  return r;
}
static void fe_store32(const fe* a, uint32_t* l) {
  for (int i = 0; i < 17; ++i) l[i] = (uint32_t)(a->w[i / 2] >> (32 * (i % 2)));
}

/* ----------------------------------------------------------- MT19937 */
typedef struct { uint32_t mt[624]; int idx; } mt_t;

static void mt_init_genrand(mt_t* s, uint32_t seed) {
  s->mt[0] = seed;
  for (int i = 1; i < 624; ++i) s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
  s->idx = 624;
}

/* CPython random.seed(int): init_by_array over the 32-bit chunks of |seed| */
static void mt_init_by_array(mt_t* s, const uint32_t* key, int len) {
  mt_init_genrand(s, 19650218u);
  int i = 1, j = 0;
  for (int k = (624 > len ? 624 : len); k; --k) {
    s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i;
    ++j;
    if (i >= 624) {
      s->mt[0] = s->mt[623];
      i = 1;
    }
    if (j >= len) j = 0;
  }
  for (int k = 623; k; --k) {
    s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= 624) {
      s->mt[0] = s->mt[623];
      i = 1;
    }
  }
  s->mt[0] = 0x80000000u;
  s->idx = 624;
}

static uint32_t mt_next(mt_t* s) {
  if (s->idx >= 624) {
    for (int k = 0; k < 624; ++k) {
      const uint32_t y = (s->mt[k] & 0x80000000u) | (s->mt[(k + 1) % 624] & 0x7fffffffu);
      s->mt[k] = s->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    s->idx = 0;
  }
  uint32_t y = s->mt[s->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

/* random.randint(1, p-1) = 1 + getrandbits(521) retried while >= p-1 */
static fe mt_randint_field(mt_t* s) {
  for (;;) {
    uint32_t l[17];
    for (int i = 0; i < 17; ++i) l[i] = mt_next(s);
    l[16] >>= 23;
    fe r = fe_load32(l);
    /* r >= p-1 = 2^521 - 2 ? */
    int ge = (r.w[8] == 0x1FF) && (r.w[0] >= 0xFFFFFFFFFFFFFFFEull);
    for (int i = 1; i < 8 && ge; ++i) ge = (r.w[i] == ~0ull);
    if (ge) continue;
    fe one = fe_from_u64(1);
    return fe_add(&r, &one);
  }
}

/* ------------------------------------------------------------ exports */

/* Seed like random.Random(seed) for 0 <= seed < 2^64, then draw n*tm1
 * coefficients (element-major), 17 u32 limbs each: out[(e*tm1 + j)*17 ...]. */
void oracle_draw_coeffs(uint64_t seed, uint64_t n, int tm1, uint32_t* out) {
  mt_t s;
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  mt_init_by_array(&s, key, (seed >> 32) ? 2 : 1);
  for (uint64_t i = 0; i < n * (uint64_t)tm1; ++i) {
    fe c = mt_randint_field(&s);
    fe_store32(&c, out + i * 17);
  }
}

/* Raw MT words after random.Random(seed) (for checking the generator). */
void oracle_mt_words(uint64_t seed, uint64_t n, uint32_t* out) {
  mt_t s;
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  mt_init_by_array(&s, key, (seed >> 32) ? 2 : 1);
  for (uint64_t i = 0; i < n; ++i) out[i] = mt_next(&s);
}

/* Split: secrets as u64 (two's-complement view of int64), coefficients
 * [n][t-1][17] u32, shares out [n_shares][n][17] u32.  _eval_at literally:
 * v = 0; for c in reversed(coeffs): v = (v*x + c) % p. */
void oracle_split(const uint64_t* secrets, const uint32_t* coeffs, uint64_t n, int t, int n_shares,
                  uint32_t* out) {
  for (uint64_t e = 0; e < n; ++e) {
    for (int x = 1; x <= n_shares; ++x) {
      fe v = fe_from_u64(0);
      const fe xf = fe_from_u64((uint64_t)x);
      for (int j = t - 1; j >= 0; --j) {
        fe c = (j == 0) ? fe_from_u64(secrets[e]) : fe_load32(coeffs + (e * (uint64_t)(t - 1) + (uint64_t)(j - 1)) * 17);
        v = fe_mul(&v, &xf);
        v = fe_add(&v, &c);
      }
      fe_store32(&v, out + ((uint64_t)(x - 1) * n + e) * 17);
    }
  }
}

/* Reconstruct (resolve_shares): ys [k][n][17], xs[k] (small, k <= 16), out [n][17].
 *   nums[i] = prod_{j!=i} (-x_j), dens[i] = prod_{j!=i} (x_i - x_j), den = prod dens
 *   num = sum_i div_mod(nums[i]*den*y_i % p, dens[i]) ; out = div_mod(num, den)  */
void oracle_reconstruct(const uint32_t* ys, const int64_t* xs, int k, uint64_t n, uint32_t* out) {
  fe nums[16], dens_inv[16], den = fe_from_u64(1);
  for (int i = 0; i < k; ++i) {
    __int128 nu = 1, de = 1;
    for (int j = 0; j < k; ++j) {
      if (j == i) continue;
      nu *= -(__int128)xs[j];
      de *= (__int128)xs[i] - (__int128)xs[j];
    }
    nums[i] = fe_from_i128(nu);
    fe d = fe_from_i128(de);
    dens_inv[i] = fe_inv(&d);
    den = fe_mul(&den, &d);
  }
  const fe den_inv = fe_inv(&den);
  for (uint64_t e = 0; e < n; ++e) {
    fe num = fe_from_u64(0);
    for (int i = 0; i < k; ++i) {
      fe y = fe_load32(ys + ((uint64_t)i * n + e) * 17);
      y = fe_reduce_wide(y.w, NL);
      fe term = fe_mul(&nums[i], &den);
      term = fe_mul(&term, &y);
      term = fe_mul(&term, &dens_inv[i]);
      num = fe_add(&num, &term);
    }
    fe r = fe_mul(&num, &den_inv);
    fe_store32(&r, out + e * 17);
  }
}
