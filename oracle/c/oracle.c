/* oracle.c — C restatement of the reference prover (CPU ORACLE; TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, as
 * the checker / the CPU baseline ("port"). The product (kzg-grandsums-study_amd/) never links it.
 *
 * Restates, op for op and with the reference's buffer-length semantics:
 *   src/grandsum/mset_eq_kzg_prover.js:12-434, src/grandsum/grandsum.js:6-62,
 *   src/grandproduct/mset_eq_kzg_prover.js:12-414, src/grandproduct/grandproduct.js:6-57,
 *   src/polynomial/polynomial.js (fromEvaluations, Lagrange1, degree, evaluate, add, sub, multiply,
 *   shiftOmega, mulScalar, addScalar, subScalar, divByXSubValue, divZh, multiExponentiation),
 *   src/polynomial/evaluations.js:12-21, src/polynomial/polynomial_utils.js, src/Keccak256Transcript.js
 * and, from their mathematical definitions, the ffjavascript@0.2.59 members they call (Montgomery
 * Fr/Fq with R = 2^256, radix-2 fft/ifft over Fr.w, batchInverse (0 -> 0), Pippenger MSM).
 * Same as the Python oracle (oracle/protocol.py), against which tests/test_oracle_c.py pins it.
 * OpenMP parallelises the NTT butterflies, the MSM windows and element-wise loops, the way
 * ffjavascript spreads fft / multiExp over its worker pool.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe;
typedef struct { uint64_t p[4], inv, one[4], r2[4]; } modp;

static const modp FR = {{0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
                        0xc2e1f593efffffffull,
                        {0xac96341c4ffffffbull, 0x36fc76959f60cd29ull, 0x666ea36f7879462eull, 0x0e0a77c19a07df2full},
                        {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull}};
static const modp FQ = {{0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
                        0x87d20782e4866389ull,
                        {0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull, 0x666ea36f7879462cull, 0x0e0a77c19a07df2full},
                        {0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull, 0x06d89f71cab8351full}};

/* ------------------------------------------------------------------ field */
static inline int geq(const uint64_t* a, const uint64_t* p) {
  for (int i = 3; i >= 0; i--) if (a[i] != p[i]) return a[i] > p[i];
  return 1;
}
static inline void subp(uint64_t* a, const uint64_t* p) {
  uint64_t b = 0;
  for (int i = 0; i < 4; i++) { u128 t = (u128)a[i] - p[i] - b; a[i] = (uint64_t)t; b = (uint64_t)(t >> 64) & 1; }
}
static inline fe f_add(const modp* M, fe a, fe b) {
  fe r; uint64_t c = 0;
  for (int i = 0; i < 4; i++) { u128 t = (u128)a.v[i] + b.v[i] + c; r.v[i] = (uint64_t)t; c = (uint64_t)(t >> 64); }
  if (geq(r.v, M->p)) subp(r.v, M->p);
  return r;
}
static inline fe f_sub(const modp* M, fe a, fe b) {
  fe r; uint64_t br = 0;
  for (int i = 0; i < 4; i++) { u128 t = (u128)a.v[i] - b.v[i] - br; r.v[i] = (uint64_t)t; br = (uint64_t)(t >> 64) & 1; }
  if (br) { uint64_t c = 0; for (int i = 0; i < 4; i++) { u128 t = (u128)r.v[i] + M->p[i] + c; r.v[i] = (uint64_t)t; c = (uint64_t)(t >> 64); } }
  return r;
}
static inline fe f_mul(const modp* M, fe a, fe b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) { u128 x = (u128)a.v[j] * b.v[i] + t[j] + c; t[j] = (uint64_t)x; c = (uint64_t)(x >> 64); }
    u128 s = (u128)t[4] + c; t[4] = (uint64_t)s; t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * M->inv;
    u128 x = (u128)m * M->p[0] + t[0]; c = (uint64_t)(x >> 64);
    for (int j = 1; j < 4; j++) { x = (u128)m * M->p[j] + t[j] + c; t[j - 1] = (uint64_t)x; c = (uint64_t)(x >> 64); }
    s = (u128)t[4] + c; t[3] = (uint64_t)s; t[4] = t[5] + (uint64_t)(s >> 64);
  }
  fe r; memcpy(r.v, t, 32);
  if (t[4] || geq(r.v, M->p)) subp(r.v, M->p);
  return r;
}
static inline int f_is0(fe a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }
static inline int f_eq(fe a, fe b) { return memcmp(a.v, b.v, 32) == 0; }
static inline fe f_zero(void) { fe r = {{0, 0, 0, 0}}; return r; }
static inline fe f_one(const modp* M) { fe r; memcpy(r.v, M->one, 32); return r; }
static inline fe f_neg(const modp* M, fe a) { return f_is0(a) ? a : f_sub(M, f_zero(), a); }
static fe f_pow(const modp* M, fe a, const uint64_t e[4]) {
  fe r = f_one(M);
  for (int i = 255; i >= 0; i--) { r = f_mul(M, r, r); if ((e[i >> 6] >> (i & 63)) & 1) r = f_mul(M, r, a); }
  return r;
}
static fe f_inv(const modp* M, fe a) { uint64_t e[4]; memcpy(e, M->p, 32); e[0] -= 2; return f_pow(M, a, e); }
static fe f_from_u64(const modp* M, uint64_t x) { fe a = {{x, 0, 0, 0}}; fe r2; memcpy(r2.v, M->r2, 32); return f_mul(M, a, r2); }
static fe f_from_std(const modp* M, const uint64_t s[4]) { fe a; memcpy(a.v, s, 32); fe r2; memcpy(r2.v, M->r2, 32); return f_mul(M, a, r2); }
static void f_to_std(const modp* M, fe a, uint64_t s[4]) { fe o = {{1, 0, 0, 0}}; fe r = f_mul(M, a, o); memcpy(s, r.v, 32); }

#define RM(a, b) f_mul(&FR, a, b)
#define RA(a, b) f_add(&FR, a, b)
#define RS(a, b) f_sub(&FR, a, b)

/* Fr.w[k]: nqr 5, s = 28 */
static fe fr_w(int k) {
  uint64_t e[4]; memcpy(e, FR.p, 32); e[0] -= 1;
  for (int s = 0; s < 28; s++) { e[0] = (e[0] >> 1) | (e[1] << 63); e[1] = (e[1] >> 1) | (e[2] << 63); e[2] = (e[2] >> 1) | (e[3] << 63); e[3] >>= 1; }
  fe w = f_pow(&FR, f_from_u64(&FR, 5), e);
  for (int s = 28; s > k; s--) w = RM(w, w);
  return w;
}

/* ------------------------------------------------------------------ NTT ([ffjs] fft / ifft) */
static int clog2(uint64_t x) { int l = 0; while ((1ull << l) < x) l++; return l; }

static void ntt(fe* a, uint64_t m, int inverse) {
  if (m <= 1) return;
  int lg = clog2(m);
  for (uint64_t i = 1, j = 0; i < m; i++) {
    uint64_t bit = m >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j |= bit;
    if (i < j) { fe t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  fe w = fr_w(lg);
  if (inverse) w = f_inv(&FR, w);
  fe* tw = (fe*)malloc(sizeof(fe) * (m / 2));
  /* tw[j] = w^j, chunked */
  const uint64_t CH = 4096;
#pragma omp parallel for schedule(static)
  for (uint64_t c = 0; c < (m / 2 + CH - 1) / CH; c++) {
    uint64_t s = c * CH, e = s + CH < m / 2 ? s + CH : m / 2;
    uint64_t ee[4] = {s, 0, 0, 0};
    fe x = f_pow(&FR, w, ee);
    for (uint64_t j = s; j < e; j++) { tw[j] = x; x = RM(x, w); }
  }
  for (uint64_t half = 1; half < m; half <<= 1) {
    const uint64_t stride = m / (2 * half);
#pragma omp parallel for schedule(static)
    for (uint64_t b = 0; b < m / 2; b++) {
      uint64_t grp = b / half, k = b % half;
      uint64_t i0 = grp * 2 * half + k, i1 = i0 + half;
      fe u = a[i0], v = RM(a[i1], tw[k * stride]);
      a[i0] = RA(u, v);
      a[i1] = RS(u, v);
    }
  }
  free(tw);
  if (inverse) {
    fe mi = f_inv(&FR, f_from_u64(&FR, m));
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < m; i++) a[i] = RM(a[i], mi);
  }
}

/* ------------------------------------------------------------------ Polynomial (polynomial.js) */
typedef struct { fe* c; uint64_t len; } poly;
static poly p_new(uint64_t len) { poly p; p.len = len; p.c = (fe*)calloc(len ? len : 1, sizeof(fe)); return p; }
static void p_free(poly* p) { free(p->c); p->c = NULL; p->len = 0; }
static poly p_clone(const poly* a) { poly p = p_new(a->len); memcpy(p.c, a->c, sizeof(fe) * a->len); return p; }
static poly p_from_evals(const fe* ev, uint64_t n) { poly p = p_new(n); memcpy(p.c, ev, sizeof(fe) * n); ntt(p.c, n, 1); return p; }
static uint64_t p_degree(const poly* a) { for (uint64_t i = a->len; i-- > 1;) if (!f_is0(a->c[i])) return i; return 0; }
static fe p_eval(const poly* a, fe x) {  /* polynomial.js:228-238 */
  fe r = f_zero();
  for (uint64_t i = p_degree(a) + 1; i > 0; i--) r = RA(a->c[i - 1], RM(r, x));
  return r;
}
static void p_addsub(poly* a, const poly* b, int sub) {  /* polynomial.js:276-350 */
  uint64_t L = a->len > b->len ? a->len : b->len;
  if (L > a->len) { a->c = (fe*)realloc(a->c, sizeof(fe) * L); memset(a->c + a->len, 0, sizeof(fe) * (L - a->len)); a->len = L; }
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < b->len; i++) a->c[i] = sub ? RS(a->c[i], b->c[i]) : RA(a->c[i], b->c[i]);
}
static void p_mul_scalar(poly* a, fe s) {
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < a->len; i++) a->c[i] = RM(a->c[i], s);
}
static void p_add_scalar(poly* a, fe s) { if (!a->len) { a->c = (fe*)realloc(a->c, sizeof(fe)); a->len = 1; a->c[0] = f_zero(); } a->c[0] = RA(a->c[0], s); }
static void p_sub_scalar(poly* a, fe s) { if (!a->len) { a->c = (fe*)realloc(a->c, sizeof(fe)); a->len = 1; a->c[0] = f_zero(); } a->c[0] = RS(a->c[0], s); }
/* Evaluations.fromPolynomial (evaluations.js:12-21): pad to 2^ceil(log2 LENGTH) * ext, fft */
static fe* evals_from_poly(const poly* a, uint64_t ext, uint64_t* outlen) {
  uint64_t L = (1ull << clog2(a->len)) * ext;
  fe* e = (fe*)calloc(L, sizeof(fe));
  memcpy(e, a->c, sizeof(fe) * a->len);
  ntt(e, L, 0);
  *outlen = L;
  return e;
}
static void p_multiply(poly* a, const poly* b) {  /* polynomial.js:352-376 */
  uint64_t da = p_degree(a), db = p_degree(b);
  int np = clog2(da + db + 1);
  uint64_t nl = 1ull << np;
  int p1 = clog2(da + 1), p2 = clog2(db + 1);
  uint64_t l1, l2;
  fe* e1 = evals_from_poly(a, 1ull << (np - p1), &l1);
  fe* e2 = evals_from_poly(b, 1ull << (np - p2), &l2);
  fe* nb = (fe*)malloc(sizeof(fe) * nl);
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < nl; i++) nb[i] = RM(e1[i], e2[i]);
  free(e1); free(e2);
  ntt(nb, nl, 1);
  free(a->c); a->c = nb; a->len = nl;
}
static void p_shift_omega(poly* a) {  /* polynomial.js:378-393 */
  uint64_t L;
  fe* e = evals_from_poly(a, 1, &L);
  fe first = e[0];
  memmove(e, e + 1, sizeof(fe) * (L - 1));
  e[L - 1] = first;
  ntt(e, L, 1);
  free(a->c); a->c = e; a->len = L;
}
static int p_div_x_sub(poly* a, fe z) {  /* polynomial.js:814-851 */
  uint64_t L = a->len;
  fe* q = (fe*)calloc(L, sizeof(fe));
  q[L - 2] = a->c[L - 1];
  for (uint64_t i = L - 2; i-- > 0;) q[i] = RA(a->c[i + 1], RM(z, q[i + 1]));
  int ok = f_eq(a->c[0], RM(f_neg(&FR, z), q[0]));
  free(a->c); a->c = q;
  return ok ? 0 : -5;
}
static int p_div_zh(poly* a, uint64_t n) {  /* polynomial.js:853-888 */
  uint64_t ext = a->len / n, deg = p_degree(a);
  uint64_t length = deg < n ? 0 : 1ull << clog2(deg + 1 - n);
  for (uint64_t i = 0; i < n; i++) a->c[i] = f_neg(&FR, a->c[i]);
  for (uint64_t i = n; i < n * ext; i++) {
    fe x = RS(a->c[i - n], a->c[i]);
    a->c[i] = x;
    if (i > n * (ext - 1) - ext && !f_is0(x)) return -4;
  }
  uint64_t d = p_degree(a);
  fe* nb = (fe*)calloc(length ? length : 1, sizeof(fe));
  memcpy(nb, a->c, sizeof(fe) * (d + 1 <= length ? d + 1 : length));
  free(a->c); a->c = nb; a->len = length;
  return 0;
}
static fe* batch_inverse(const fe* v, uint64_t n) {  /* [ffjs] Fr.batchInverse, 0 -> 0 */
  fe* out = (fe*)malloc(sizeof(fe) * n);
  fe acc = f_one(&FR);
  for (uint64_t i = 0; i < n; i++) { out[i] = acc; if (!f_is0(v[i])) acc = RM(acc, v[i]); }
  fe inv = f_inv(&FR, acc);
  for (uint64_t i = n; i-- > 0;) {
    if (f_is0(v[i])) { out[i] = f_zero(); continue; }
    out[i] = RM(inv, out[i]);
    inv = RM(inv, v[i]);
  }
  return out;
}

/* ------------------------------------------------------------------ G1 + MSM */
typedef struct { fe X, Y, ZZ, ZZZ; } g1;
#define QM(a, b) f_mul(&FQ, a, b)
#define QA(a, b) f_add(&FQ, a, b)
#define QS(a, b) f_sub(&FQ, a, b)
static g1 g_inf(void) { g1 r; r.X = f_one(&FQ); r.Y = f_one(&FQ); r.ZZ = f_zero(); r.ZZZ = f_zero(); return r; }
static g1 g_dbl(g1 p) {
  if (f_is0(p.ZZ)) return p;
  fe U = QA(p.Y, p.Y), V = QM(U, U), W = QM(U, V), S = QM(p.X, V), X2 = QM(p.X, p.X);
  fe M = QA(QA(X2, X2), X2);
  g1 r;
  r.X = QS(QM(M, M), QA(S, S));
  r.Y = QS(QM(M, QS(S, r.X)), QM(W, p.Y));
  r.ZZ = QM(V, p.ZZ);
  r.ZZZ = QM(W, p.ZZZ);
  return r;
}
static g1 g_add(g1 p, g1 q) {
  if (f_is0(q.ZZ)) return p;
  if (f_is0(p.ZZ)) return q;
  fe U1 = QM(p.X, q.ZZ), U2 = QM(q.X, p.ZZ), S1 = QM(p.Y, q.ZZZ), S2 = QM(q.Y, p.ZZZ);
  fe P = QS(U2, U1), R = QS(S2, S1);
  if (f_is0(P)) return f_is0(R) ? g_dbl(p) : g_inf();
  fe PP = QM(P, P), PPP = QM(P, PP), Qv = QM(U1, PP);
  g1 r;
  r.X = QS(QS(QM(R, R), PPP), QA(Qv, Qv));
  r.Y = QS(QM(R, QS(Qv, r.X)), QM(S1, PPP));
  r.ZZ = QM(QM(p.ZZ, q.ZZ), PP);
  r.ZZZ = QM(QM(p.ZZZ, q.ZZZ), PPP);
  return r;
}
static g1 g_madd(g1 p, fe x, fe y) {  /* p + affine (x,y); (0,0) = infinity */
  if (f_is0(x) && f_is0(y)) return p;
  if (f_is0(p.ZZ)) { g1 r; r.X = x; r.Y = y; r.ZZ = f_one(&FQ); r.ZZZ = f_one(&FQ); return r; }
  fe U2 = QM(x, p.ZZ), S2 = QM(y, p.ZZZ), P = QS(U2, p.X), R = QS(S2, p.Y);
  if (f_is0(P)) {
    if (!f_is0(R)) return g_inf();
    g1 a; a.X = x; a.Y = y; a.ZZ = f_one(&FQ); a.ZZZ = f_one(&FQ);
    return g_dbl(a);
  }
  fe PP = QM(P, P), PPP = QM(P, PP), Qv = QM(p.X, PP);
  g1 r;
  r.X = QS(QS(QM(R, R), PPP), QA(Qv, Qv));
  r.Y = QS(QM(R, QS(Qv, r.X)), QM(p.Y, PPP));
  r.ZZ = QM(p.ZZ, PP);
  r.ZZZ = QM(p.ZZZ, PPP);
  return r;
}
static void g_affine(g1 p, uint8_t out[64]) {
  if (f_is0(p.ZZ)) { memset(out, 0, 64); return; }
  fe inv = f_inv(&FQ, QM(p.ZZ, p.ZZZ));
  fe x = QM(p.X, QM(inv, p.ZZZ)), y = QM(p.Y, QM(inv, p.ZZ));
  memcpy(out, x.v, 32);
  memcpy(out + 32, y.v, 32);
}
/* [ffjs] G1.multiExpAffine: unsigned-window Pippenger, windows in parallel */
static void msm(const uint8_t* bases, const fe* sc_mont, uint64_t n, uint8_t out[64]) {
  if (n == 0) { memset(out, 0, 64); return; }
  uint64_t (*s)[4] = malloc(sizeof(uint64_t[4]) * n);
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; i++) f_to_std(&FR, sc_mont[i], s[i]);
  int c = clog2(n) - 3;
  if (c < 2) c = 2;
  if (c > 16) c = 16;
  const int nw = (254 + c - 1) / c;
  g1* wsum = (g1*)malloc(sizeof(g1) * nw);
#pragma omp parallel for schedule(dynamic, 1)
  for (int w = 0; w < nw; w++) {
    g1* bk = (g1*)malloc(sizeof(g1) * (1u << c));
    for (uint32_t b = 0; b < (1u << c); b++) bk[b] = g_inf();
    const int bit = w * c;
    for (uint64_t i = 0; i < n; i++) {
      uint32_t d = 0;
      for (int k = 0; k < c && bit + k < 256; k++) d |= (uint32_t)((s[i][(bit + k) >> 6] >> ((bit + k) & 63)) & 1) << k;
      if (!d) continue;
      fe x, y;
      memcpy(x.v, bases + 64 * i, 32);
      memcpy(y.v, bases + 64 * i + 32, 32);
      bk[d] = g_madd(bk[d], x, y);
    }
    g1 run = g_inf(), acc = g_inf();
    for (uint32_t b = (1u << c) - 1; b > 0; b--) { run = g_add(run, bk[b]); acc = g_add(acc, run); }
    wsum[w] = acc;
    free(bk);
  }
  g1 tot = g_inf();
  for (int w = nw - 1; w >= 0; w--) {
    for (int k = 0; k < c; k++) tot = g_dbl(tot);
    tot = g_add(tot, wsum[w]);
  }
  g_affine(tot, out);
  free(wsum);
  free(s);
}
/* polynomial.js:1106-1115: N = degree()+1 */
static void commit(const poly* p, const uint8_t* srs, uint8_t out[64]) { msm(srs, p->c, p_degree(p) + 1, out); }

/* ------------------------------------------------------------------ keccak + transcript */
static void keccakf(uint64_t s[25]) {
  static const uint64_t RC[24] = {0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
      0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull, 0x000000000000008Aull,
      0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull, 0x000000008000808Bull, 0x800000000000008Bull,
      0x8000000000008089ull, 0x8000000000008003ull, 0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull,
      0x800000008000000Aull, 0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
  static const int rho[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
  static const int pi[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
  for (int r = 0; r < 24; r++) {
    uint64_t C[5];
    for (int x = 0; x < 5; x++) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
    for (int x = 0; x < 5; x++) {
      uint64_t D = C[(x + 4) % 5] ^ ((C[(x + 1) % 5] << 1) | (C[(x + 1) % 5] >> 63));
      for (int y = 0; y < 25; y += 5) s[y + x] ^= D;
    }
    uint64_t t = s[1];
    for (int i = 0; i < 24; i++) {
      int j = pi[i];
      uint64_t tmp = s[j];
      s[j] = (t << rho[i]) | (t >> (64 - rho[i]));
      t = tmp;
    }
    for (int y = 0; y < 25; y += 5) {
      uint64_t b[5];
      for (int x = 0; x < 5; x++) b[x] = s[y + x];
      for (int x = 0; x < 5; x++) s[y + x] = b[x] ^ ((~b[(x + 1) % 5]) & b[(x + 2) % 5]);
    }
    s[0] ^= RC[r];
  }
}
void orc_keccak256(const uint8_t* data, uint64_t len, uint8_t out[32]) {
  uint64_t s[25];
  memset(s, 0, sizeof(s));
  uint8_t blk[136];
  uint64_t off = 0;
  for (;;) {
    uint64_t take = len - off < 136 ? len - off : 136;
    memset(blk, 0, 136);
    memcpy(blk, data + off, take);
    int last = take < 136;
    if (last) { blk[take] |= 0x01; blk[135] |= 0x80; }
    for (int i = 0; i < 17; i++) { uint64_t w; memcpy(&w, blk + 8 * i, 8); s[i] ^= w; }
    keccakf(s);
    off += take;
    if (last) break;
  }
  memcpy(out, s, 32);
}
typedef struct { uint8_t* buf; uint64_t len, cap; } transcript;
static void tr_push(transcript* t, const uint8_t* d, uint64_t n) {
  if (t->len + n > t->cap) { t->cap = (t->len + n) * 2 + 256; t->buf = (uint8_t*)realloc(t->buf, t->cap); }
  memcpy(t->buf + t->len, d, n);
  t->len += n;
}
static void be_std(const modp* M, fe a, uint8_t out[32]) {
  uint64_t s[4];
  f_to_std(M, a, s);
  for (int i = 0; i < 4; i++) for (int k = 0; k < 8; k++) out[(3 - i) * 8 + k] = (uint8_t)(s[i] >> (56 - 8 * k));
}
static void tr_commit(transcript* t, const uint8_t lem[64]) {  /* G1.toRprUncompressed */
  uint8_t o[64];
  fe x, y;
  memcpy(x.v, lem, 32);
  memcpy(y.v, lem + 32, 32);
  if (f_is0(x) && f_is0(y)) { memset(o, 0, 64); o[0] = 0x40; }
  else { be_std(&FQ, x, o); be_std(&FQ, y, o + 32); }
  tr_push(t, o, 64);
}
static void tr_scalar(transcript* t, fe s) { uint8_t o[32]; be_std(&FR, s, o); tr_push(t, o, 32); }
static fe tr_challenge(const transcript* t) {
  uint8_t h[32];
  orc_keccak256(t->buf, t->len, h);
  uint64_t s[4];
  for (int i = 0; i < 4; i++) { uint64_t w = 0; for (int k = 0; k < 8; k++) w = (w << 8) | h[(3 - i) * 8 + k]; s[i] = w; }
  while (geq(s, FR.p)) subp(s, FR.p);
  return f_from_std(&FR, s);
}

/* ------------------------------------------------------------------ provers */
/* kind 0 = grand-sum, 1 = grand-product, 2 = lookup (grand-sum with selt = multiplicities and no
 * binary constraint on selt; selectors required). Outputs in the C-ABI order of include/kgs.h.
 * Returns 0 or -3 (not well calculated), -4 (not divisible), -5 (does not divide), -1 (args). */
int orc_prove(int kind, int nbits, int npols, const uint8_t* const* f_std, const uint8_t* const* t_std,
              const uint8_t* self, const uint8_t* selt, const uint8_t* srs, uint64_t npts, int threads,
              uint8_t* com_out, uint8_t* ev_out) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  if (npols < 1 || nbits < 1 || kind < 0 || kind > 2) return -1;
  if (kind == 2 && (!self || !selt)) return -1;
  const int gs = kind != 1, lk = kind == 2, sel = self != NULL, vec = npols > 1;
  const uint64_t n = 1ull << nbits;
  if (npts < 2 * n - 1) return -1;
  const fe one = f_one(&FR);
  int rc = 0;
  poly* Fp = (poly*)calloc(npols, sizeof(poly));
  poly* Tp = (poly*)calloc(npols, sizeof(poly));
  fe** fev = (fe**)calloc(npols, sizeof(fe*));
  fe** tev = (fe**)calloc(npols, sizeof(fe*));
  uint8_t(*com)[64] = malloc(64 * (2 * npols + 8));
  int nc = 0;
  /* round 1 */
  for (int i = 0; i < npols; i++) {
    fev[i] = (fe*)malloc(sizeof(fe) * n);
    tev[i] = (fe*)malloc(sizeof(fe) * n);
#pragma omp parallel for schedule(static)
    for (uint64_t j = 0; j < n; j++) {
      uint64_t a[4], b[4];
      memcpy(a, f_std[i] + 32 * j, 32);
      memcpy(b, t_std[i] + 32 * j, 32);
      fev[i][j] = f_from_std(&FR, a);
      tev[i][j] = f_from_std(&FR, b);
    }
    Fp[i] = p_from_evals(fev[i], n);
    Tp[i] = p_from_evals(tev[i], n);
  }
  for (int i = 0; i < npols; i++) { commit(&Fp[i], srs, com[nc++]); commit(&Tp[i], srs, com[nc++]); }
  fe *sfv = (fe*)malloc(sizeof(fe) * n), *stv = (fe*)malloc(sizeof(fe) * n);
  for (uint64_t j = 0; j < n; j++) {
    if (sel) { memcpy(sfv[j].v, self + 32 * j, 32); memcpy(stv[j].v, selt + 32 * j, 32); }
    else { sfv[j] = one; stv[j] = one; }
  }
  poly selF = {0}, selT = {0};
  if (sel) {
    selF = p_from_evals(sfv, n);
    selT = p_from_evals(stv, n);
    commit(&selF, srs, com[nc++]);
    commit(&selT, srs, com[nc++]);
  }
  /* round 2 */
  transcript tr = {0};
  for (int i = 0; i < nc; i++) tr_commit(&tr, com[i]);
  fe beta = f_zero();
  if (vec) { beta = tr_challenge(&tr); tr_scalar(&tr, beta); }
  fe gamma = tr_challenge(&tr);
  poly polF, polT;
  fe *evF, *evT;
  int own = 0;
  if (vec) {
    polF = p_new(n);
    polT = p_new(n);
    for (int i = npols - 1; i >= 0; i--) {
      p_mul_scalar(&polF, beta); p_addsub(&polF, &Fp[i], 0);
      p_mul_scalar(&polT, beta); p_addsub(&polT, &Tp[i], 0);
    }
    uint64_t L;
    evF = evals_from_poly(&polF, 1, &L);
    evT = evals_from_poly(&polT, 1, &L);
    own = 1;
  } else {
    polF = Fp[0];
    polT = Tp[0];
    evF = fev[0];
    evT = tev[0];
  }
  fe* num = (fe*)malloc(sizeof(fe) * n);
  fe* den = (fe*)malloc(sizeof(fe) * n);
  num[0] = gs ? f_zero() : one;
  den[0] = gs ? f_zero() : one;
  for (uint64_t i = 0; i < n; i++) {
    fe f = RA(evF[i], gamma), t = RA(evT[i], gamma);
    uint64_t j = (i + 1) % n;
    if (gs) { num[j] = RS(RM(t, sfv[i]), RM(f, stv[i])); den[j] = RM(f, t); }
    else { num[j] = RA(RM(sfv[i], RS(f, one)), one); den[j] = RA(RM(stv[i], RS(t, one)), one); }
  }
  fe* dinv = batch_inverse(den, n);
  fe last = gs ? f_zero() : one;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t j = (i + 1) % n;
    fe s = RM(num[j], dinv[j]);
    last = gs ? RA(s, last) : RM(s, last);
    num[j] = last;
  }
  free(dinv); free(den);
  if (gs ? !f_is0(num[0]) : !f_eq(num[0], one)) { rc = -3; free(num); goto done; }
  poly polS = p_from_evals(num, n);
  free(num);
  const int iS = nc;
  commit(&polS, srs, com[nc++]);
  /* round 3 */
  tr_scalar(&tr, gamma);
  tr_commit(&tr, com[iS]);
  fe alpha = tr_challenge(&tr);
  poly polQ = p_new(n);
  if (sel) {
    poly b1, b2, sb;
    if (!lk) { /* prover.js:241-244 (a lookup's selT holds multiplicities) */
      b1 = p_clone(&selT); b2 = p_clone(&selT); p_multiply(&b1, &b2);
      sb = p_clone(&selT); p_addsub(&sb, &b1, 1); p_addsub(&polQ, &sb, 0);
      p_free(&b1); p_free(&b2); p_free(&sb);
    }
    p_mul_scalar(&polQ, alpha);
    b1 = p_clone(&selF); b2 = p_clone(&selF); p_multiply(&b1, &b2);
    sb = p_clone(&selF); p_addsub(&sb, &b1, 1); p_addsub(&polQ, &sb, 0); p_mul_scalar(&polQ, alpha);
    p_free(&b1); p_free(&b2); p_free(&sb);
  }
  poly Q1 = p_clone(&polS);
  p_shift_omega(&Q1);
  poly FG = p_clone(&polF), TG = p_clone(&polT);
  p_add_scalar(&FG, gamma);
  p_add_scalar(&TG, gamma);
  poly L1 = {0};
  {
    fe* e = (fe*)calloc(n, sizeof(fe));
    e[0] = one;
    L1 = p_from_evals(e, n);
    free(e);
  }
  if (gs) {
    p_addsub(&Q1, &polS, 1);
    p_multiply(&Q1, &FG);
    p_multiply(&Q1, &TG);
    if (sel) {
      poly a = p_clone(&selF); p_multiply(&a, &TG);
      poly b = p_clone(&selT); p_multiply(&b, &FG);
      p_addsub(&Q1, &b, 0); p_addsub(&Q1, &a, 1);
      p_free(&a); p_free(&b);
    } else {
      p_addsub(&Q1, &polF, 0); p_addsub(&Q1, &polT, 1);
    }
    p_addsub(&polQ, &Q1, 0); p_mul_scalar(&polQ, alpha);
    poly Q2 = p_clone(&polS); p_multiply(&Q2, &L1); p_addsub(&polQ, &Q2, 0); p_free(&Q2);
  } else {
    poly Q2 = p_clone(&polS);
    if (sel) {
      poly st = p_clone(&selT), sf = p_clone(&selF);
      p_sub_scalar(&TG, one); p_multiply(&TG, &st); p_add_scalar(&TG, one); p_multiply(&Q1, &TG);
      p_sub_scalar(&FG, one); p_multiply(&FG, &sf); p_add_scalar(&FG, one); p_multiply(&Q2, &FG);
      p_free(&st); p_free(&sf);
    } else {
      p_multiply(&Q1, &TG);
      p_multiply(&Q2, &FG);
    }
    p_addsub(&Q1, &Q2, 1);
    p_addsub(&polQ, &Q1, 0); p_mul_scalar(&polQ, alpha);
    poly Q3 = p_clone(&polS); p_sub_scalar(&Q3, one); p_multiply(&Q3, &L1); p_addsub(&polQ, &Q3, 0); p_free(&Q3);
    p_free(&Q2);
  }
  p_free(&Q1); p_free(&FG); p_free(&TG); p_free(&L1);
  if (p_div_zh(&polQ, n)) { rc = -4; goto done2; }
  const int iQ = nc;
  commit(&polQ, srs, com[nc++]);
  /* round 4 */
  tr_scalar(&tr, alpha);
  tr_commit(&tr, com[iQ]);
  fe xi = tr_challenge(&tr);
  fe w = fr_w(nbits), xiw = RM(xi, w);
  fe* ev = (fe*)malloc(sizeof(fe) * (2 * npols + 3));
  int ne = 0;
  fe *fx = (fe*)malloc(sizeof(fe) * npols), *tx = (fe*)malloc(sizeof(fe) * npols);
  for (int i = 0; i < npols; i++) {
    fx[i] = p_eval(&Fp[i], xi); ev[ne++] = fx[i];
    if (gs) { tx[i] = p_eval(&Tp[i], xi); ev[ne++] = tx[i]; }
  }
  fe sFx = f_zero(), sTx = f_zero();
  if (sel) { sFx = p_eval(&selF, xi); sTx = p_eval(&selT, xi); ev[ne++] = sFx; ev[ne++] = sTx; }
  fe sxiw = p_eval(&polS, xiw);
  ev[ne++] = sxiw;
  /* round 5 */
  tr_scalar(&tr, xi);
  for (int i = 0; i < npols; i++) { tr_scalar(&tr, fx[i]); if (gs) tr_scalar(&tr, tx[i]); }
  if (sel) { tr_scalar(&tr, sFx); tr_scalar(&tr, sTx); }
  tr_scalar(&tr, sxiw);
  fe v = tr_challenge(&tr);
  fe xn = xi;
  for (int i = 0; i < nbits; i++) xn = RM(xn, xn);
  fe zh = RS(xn, one);
  fe l1 = RM(zh, f_inv(&FR, RM(f_from_u64(&FR, n), RS(xi, one))));
  poly polR = p_new(n);
  if (sel) {
    if (!lk) p_add_scalar(&polR, RS(sTx, RM(sTx, sTx)));
    p_mul_scalar(&polR, alpha);
    p_add_scalar(&polR, RS(sFx, RM(sFx, sFx))); p_mul_scalar(&polR, alpha);
  }
  fe fxi = p_eval(&polF, xi);
  if (gs) {
    poly R1 = p_clone(&polS);
    p_mul_scalar(&R1, f_neg(&FR, one)); p_add_scalar(&R1, sxiw);
    fe txi = p_eval(&polT, xi);
    fe fg = RA(fxi, gamma), tg = RA(txi, gamma);
    p_mul_scalar(&R1, fg); p_mul_scalar(&R1, tg);
    if (sel) { p_add_scalar(&R1, RM(sTx, fg)); p_sub_scalar(&R1, RM(sFx, tg)); }
    else { p_add_scalar(&R1, fxi); p_sub_scalar(&R1, txi); }
    p_addsub(&polR, &R1, 0); p_mul_scalar(&polR, alpha);
    poly R2 = p_clone(&polS); p_mul_scalar(&R2, l1); p_addsub(&polR, &R2, 0);
    p_free(&R1); p_free(&R2);
  } else {
    poly R1 = p_new(n);
    fe fg = RA(fxi, gamma);
    poly tgp = p_clone(&polT); p_add_scalar(&tgp, gamma);  /* prover.js:353 mutates polT: no value effect */
    if (sel) {
      fg = RS(fg, one);
      p_sub_scalar(&tgp, one);
      fe sfg = RA(RM(sFx, fg), one);
      p_mul_scalar(&tgp, sTx); p_add_scalar(&tgp, one);
      p_mul_scalar(&tgp, sxiw);
      p_addsub(&R1, &tgp, 0);
      poly ZZ = p_clone(&polS); p_mul_scalar(&ZZ, sfg); p_addsub(&R1, &ZZ, 1); p_free(&ZZ);
    } else {
      p_mul_scalar(&tgp, sxiw);
      p_addsub(&R1, &tgp, 0);
      poly ZZ = p_clone(&polS); p_mul_scalar(&ZZ, fg); p_addsub(&R1, &ZZ, 1); p_free(&ZZ);
    }
    p_addsub(&polR, &R1, 0); p_mul_scalar(&polR, alpha);
    poly R2 = p_clone(&polS); p_sub_scalar(&R2, one); p_mul_scalar(&R2, l1); p_addsub(&polR, &R2, 0);
    p_free(&R1); p_free(&R2); p_free(&tgp);
  }
  {
    poly R3 = p_clone(&polQ); p_mul_scalar(&R3, zh); p_addsub(&polR, &R3, 1); p_free(&R3);
  }
  poly W = p_new(n);
  if (sel) {
    poly a = p_clone(&selT); p_sub_scalar(&a, sTx); p_addsub(&W, &a, 0); p_free(&a);
    p_mul_scalar(&W, v);
    a = p_clone(&selF); p_sub_scalar(&a, sFx); p_addsub(&W, &a, 0); p_free(&a);
  }
  if (gs)
    for (int i = npols - 1; i >= 0; i--) {
      p_mul_scalar(&W, v);
      poly a = p_clone(&Tp[i]); p_sub_scalar(&a, tx[i]); p_addsub(&W, &a, 0); p_free(&a);
    }
  for (int i = npols - 1; i >= 0; i--) {
    p_mul_scalar(&W, v);
    poly a = p_clone(&Fp[i]); p_sub_scalar(&a, fx[i]); p_addsub(&W, &a, 0); p_free(&a);
  }
  p_mul_scalar(&W, v);
  p_addsub(&W, &polR, 0);
  int e1 = p_div_x_sub(&W, xi);
  poly Ww = p_clone(&polS);
  p_sub_scalar(&Ww, sxiw);
  int e2 = p_div_x_sub(&Ww, xiw);
  if (e1 || e2) rc = -5;
  else {
    commit(&W, srs, com[nc++]);
    commit(&Ww, srs, com[nc++]);
    memcpy(com_out, com, 64 * (size_t)nc);
    for (int i = 0; i < ne; i++) memcpy(ev_out + 32 * i, ev[i].v, 32);
  }
  p_free(&W); p_free(&Ww); p_free(&polR);
  free(ev); free(fx); free(tx);
done2:
  p_free(&polQ);
  p_free(&polS);
done:
  if (own) { p_free(&polF); p_free(&polT); free(evF); free(evT); }
  for (int i = 0; i < npols; i++) { p_free(&Fp[i]); p_free(&Tp[i]); free(fev[i]); free(tev[i]); }
  if (sel) { p_free(&selF); p_free(&selT); }
  free(Fp); free(Tp); free(fev); free(tev); free(sfv); free(stv); free(com); free(tr.buf);
  return rc;
}

/* single MSM (N scalars, Montgomery) over the given bases, for tests */
void orc_msm(const uint8_t* bases, const uint8_t* sc_mont, uint64_t n, int threads, uint8_t out[64]) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  msm(bases, (const fe*)sc_mont, n, out);
}

int orc_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* p(x) from the evaluations of p on <w_n> (natural order), standard-form 32 B LE in and out:
 * p(x) = (x^n - 1)/n * sum_i e_i w^i / (x - w^i) (barycentric; x not in <w_n>). Test checker for the
 * transcript-independent commitments of large proofs: C(F) == F(tau) G1 (tests/test_gpu_configs.py).
 * Chunked Montgomery batch inversion, one chunk per thread. */
/* NTT of m = 2^k Montgomery elements in place, natural order in and out ([ffjs] Fr.fft / Fr.ifft,
 * polynomial.js:34,373,392): the checker of the GPU transforms at sizes the Python oracle is too slow for */
void orc_ntt(uint8_t* data_mont, uint64_t m, int inverse, int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  fe* a = (fe*)malloc(sizeof(fe) * (m ? m : 1));
  memcpy(a, data_mont, 32 * m);
  ntt(a, m, inverse);
  memcpy(data_mont, a, 32 * m);
  free(a);
}

int orc_eval_evals_std(const uint8_t* evals_std, int nbits, const uint8_t x_std[32], uint8_t out_std[32]) {
  const uint64_t n = 1ull << nbits;
  uint64_t xs[4];
  memcpy(xs, x_std, 32);
  const fe x = f_from_std(&FR, xs);
  const fe w = fr_w(nbits);
  int nth = 1;
#ifdef _OPENMP
  nth = omp_get_max_threads();
#endif
  if ((uint64_t)nth > n) nth = (int)n;
  fe* part = (fe*)calloc(nth, sizeof(fe));
  int bad = 0;
#ifdef _OPENMP
#pragma omp parallel num_threads(nth) reduction(| : bad)
#endif
  {
    int t = 0;
#ifdef _OPENMP
    t = omp_get_thread_num();
#endif
    const uint64_t lo = n * t / nth, hi = n * (t + 1) / nth, m = hi - lo;
    uint64_t e[4] = {lo, 0, 0, 0};
    fe wi = f_pow(&FR, w, e);  /* w^lo */
    fe* den = (fe*)malloc(sizeof(fe) * (m ? m : 1));
    fe* wp = (fe*)malloc(sizeof(fe) * (m ? m : 1));
    for (uint64_t i = 0; i < m; i++) {
      wp[i] = wi;
      den[i] = RS(x, wi);
      if (f_is0(den[i])) bad = 1;
      wi = RM(wi, w);
    }
    if (m == 0) den[0] = f_zero();
    fe* inv = batch_inverse(den, m);
    fe s = f_zero();
    for (uint64_t i = 0; i < m; i++) {
      uint64_t v[4];
      memcpy(v, evals_std + 32 * (lo + i), 32);
      s = RA(s, RM(RM(f_from_std(&FR, v), wp[i]), inv[i]));
    }
    part[t] = s;
    free(den); free(wp); free(inv);
  }
  if (bad) { free(part); return -1; }
  fe s = f_zero();
  for (int t = 0; t < nth; t++) s = RA(s, part[t]);
  free(part);
  uint64_t en[4] = {n, 0, 0, 0};
  fe xn = f_pow(&FR, x, en);
  fe scale = RM(RS(xn, f_one(&FR)), f_inv(&FR, f_from_u64(&FR, n)));
  fe r = RM(scale, s);
  uint64_t o[4];
  f_to_std(&FR, r, o);
  memcpy(out_std, o, 32);
  return 0;
}
