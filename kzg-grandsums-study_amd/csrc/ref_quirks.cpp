// Reference-quirks mode (kgs_ctx_set_reference_quirks, KGS_REFERENCE_QUIRKS=1): the reference's own
// quotient chain (src/grandsum/mset_eq_kzg_prover.js:233-286, src/grandproduct/mset_eq_kzg_prover.js:
// 233-286) replayed on the GPU with the reference's buffer semantics, for the degenerate inputs on
// which the reference does not compute the mathematical quotient (DESIGN.md §4 "Reference quirks"):
//   Q1 Polynomial.multiply (polynomial.js:352-376) sizes an operand's transform from its degree but
//      Evaluations.fromPolynomial (evaluations.js:12-18) pads from its buffer length: an operand of
//      degree 1 <= d < length/2 is evaluated on the first N points of a larger domain — a product
//      that is not the product;
//   Q2 add / sub (polynomial.js:276-350) with a strictly longer argument write into the argument's
//      buffer and adopt it, so two objects share one buffer afterwards;
//   Q3 divZh (polynomial.js:853-888) copies degree()+1 coefficients into a buffer of 0 elements when
//      the dividend's degree is below n: V8 throws "RangeError: offset is out of bounds".
// The default (fast) path computes the mathematical quotient on a coset instead; on every input
// where no base operand (F, T, S, selF, selT) has degree 1 <= d < n/2 the two agree except for Q3,
// which the fast path detects from its own quotient (Q == 0 <=> dividend of degree < n). Only when
// some operand has such a degree is the chain replayed, op for op, with device buffers.
#include <memory>
#include <string>
#include <vector>

#include "context.hpp"

namespace kgsi {

namespace {

int clog2(uint64_t x) {  // Math.ceil(Math.log2(x)), x >= 1
  int l = 0;
  while ((1ull << l) < x) l++;
  return l;
}

// largest transform the replay runs (2^26 points: 2 GiB per operand; the reference would need more)
constexpr int REF_LOG_MAX = 26;

struct RefBuf {
  uint32_t* p = nullptr;
  uint64_t len = 0;  // elements
  int device = 0;
  bool written = false;  // written in place (by its own object or, shared, by another: Q2)
  ~RefBuf() {
    if (p) {
      hipSetDevice(device);
      hipFree(p);
    }
  }
};
using BufP = std::shared_ptr<RefBuf>;

// a reference Polynomial object: `coef` may be shared with another object (Q2)
struct RPoly {
  BufP b;
  uint64_t len() const { return b->len; }
};

struct Engine {
  kgs_ctx& c;
  hipStream_t st;
  uint32_t* d_scratch;  // degree / flag words
  uint32_t* h_scratch;
  // every buffer of the replay stays allocated until the stream has drained (~Engine), whatever
  // object still refers to it
  std::vector<BufP> keep;

  explicit Engine(kgs_ctx& cc) : c(cc), st(cc.st) {
    d_scratch = c.buf("refq_scratch", 64);
    h_scratch = (uint32_t*)c.pin(64);
  }
  ~Engine() {
    hipStreamSynchronize(st);
    keep.clear();
  }

  BufP alloc(uint64_t len) {
    auto b = std::make_shared<RefBuf>();
    b->device = c.device;
    b->len = len;
    HC(dev_malloc((void**)&b->p, 32 * (len ? len : 1)));
    keep.push_back(b);
    return b;
  }
  RPoly wrap(const uint32_t* src, uint64_t len) {  // a copy of one of the prover's buffers
    RPoly r{alloc(len)};
    HC(hipMemcpyAsync(r.b->p, src, 32 * len, hipMemcpyDeviceToDevice, st));
    return r;
  }
  RPoly zero(uint64_t len) {  // Polynomial.zero (polynomial.js:63-66)
    RPoly r{alloc(len)};
    HC(hipMemsetAsync(r.b->p, 0, 32 * len, st));
    return r;
  }
  RPoly clone(const RPoly& a) { return wrap(a.b->p, a.len()); }  // polynomial.js:80-82

  uint64_t degree(const RPoly& a) {  // polynomial.js:212-226
    HC(hipMemsetAsync(d_scratch, 0, 4, st));
    launch_degree(st, d_scratch, a.b->p, a.len());
    check_launch();
    HC(hipMemcpyAsync(h_scratch, d_scratch, 4, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    return h_scratch[0];
  }

  void mul_scalar(RPoly& a, const Fr& k) {  // polynomial.js:395-406, in place
    a.b->written = true;
    LcTerms t;
    t.add(a.b->p, a.len(), k);
    run_lincomb(st, a.b->p, a.len(), t);
  }
  void add_scalar(RPoly& a, const Fr& k) {  // polynomial.js:408-422, coefficient 0 in place
    if (a.len() == 0) throw KgsError(KGS_E_RANGE, "offset is out of bounds");
    a.b->written = true;
    LcTerms t;
    t.add(a.b->p, 1, Fr::one());
    t.c0 = k;
    run_lincomb(st, a.b->p, 1, t);
  }
  // add / sub (polynomial.js:276-350): into self's buffer, or — the argument strictly longer — into
  // the argument's buffer, which self then adopts (Q2)
  void addsub(RPoly& self, RPoly& other, bool sub) {
    const Fr s = sub ? Fr::one().neg() : Fr::one();
    LcTerms t;
    if (other.len() > self.len()) {
      other.b->written = true;
      t.add(self.b->p, self.len(), Fr::one());
      t.add(other.b->p, other.len(), s);
      run_lincomb(st, other.b->p, other.len(), t);
      self.b = other.b;
    } else {
      self.b->written = true;
      t.add(self.b->p, self.len(), Fr::one());
      t.add(other.b->p, other.len(), s);
      run_lincomb(st, self.b->p, self.len(), t);
    }
  }
  RPoly& add(RPoly& self, RPoly&& o) { addsub(self, o, false); return self; }
  RPoly& add(RPoly& self, RPoly& o) { addsub(self, o, false); return self; }
  RPoly& sub(RPoly& self, RPoly&& o) { addsub(self, o, true); return self; }
  RPoly& sub(RPoly& self, RPoly& o) { addsub(self, o, true); return self; }

  void need_domain(int logm) {
    if (logm > REF_LOG_MAX)
      throw KgsError(KGS_E_ARG, "reference-quirks mode: the reference's Polynomial.multiply would evaluate an operand on 2^" +
                                    std::to_string(logm) +
                                    " points here (polynomial.js:352-376, evaluations.js:12-18); the replay stops at 2^" +
                                    std::to_string(REF_LOG_MAX));
    if (logm > c.logM) {
      HC(hipStreamSynchronize(st));
      ensure_domain(c, logm, false);  // replay-only growth: no 29-bit twin
    }
  }
  // Evaluations.fromPolynomial(a, factor) (evaluations.js:12-18): a zero-padded to 2^logB, forward
  // transform, left in bit-reversed order (the gather reads it there). A constant operand (degree 0)
  // has the same value at every point: its coefficient 0 stands for the whole transform.
  BufP transform(const RPoly& a, uint64_t deg, int logB, int& log_out) {
    if (deg == 0) {
      log_out = 0;
      return a.b;
    }
    need_domain(logB);
    BufP e = alloc(1ull << logB);
    ntt_dif(st, e->p, a.b->p, a.len(), logB, nullptr, c.tw_fwd, c.logM);
    check_launch();
    log_out = logB;
    return e;
  }
  // Polynomial.multiply (polynomial.js:352-376) with the reference's sizes (Q1)
  void multiply(RPoly& self, const RPoly& other) {
    const uint64_t d1 = degree(self), d2 = degree(other);
    const int np = clog2(d1 + d2 + 1);
    const uint64_t N = 1ull << np;
    const int lb1 = clog2(self.len()) + np - clog2(d1 + 1);
    const int lb2 = clog2(other.len()) + np - clog2(d2 + 1);
    int l1 = 0, l2 = 0;
    BufP e1 = transform(self, d1, lb1, l1);
    BufP e2 = transform(other, d2, lb2, l2);
    need_domain(np);
    BufP prod = alloc(N);
    launch_ref_gather_mul(st, prod->p, e1->p, l1, e2->p, l2, N, 0);
    BufP out = alloc(N);
    intt_nat(c, out->p, prod->p, np, st);
    check_launch();
    self.b = out;  // this.coef = newCoefs
  }
  // Polynomial.shiftOmega (polynomial.js:378-393): transform of size 2^ceil(log2(length)), rotate
  // by one, inverse transform
  void shift_omega(RPoly& self) {
    const int lg = clog2(self.len());
    need_domain(lg);
    BufP e = alloc(1ull << lg);
    ntt_dif(st, e->p, self.b->p, self.len(), lg, nullptr, c.tw_fwd, c.logM);
    BufP rot = alloc(1ull << lg);
    launch_ref_gather_mul(st, rot->p, e->p, lg, nullptr, 0, 1ull << lg, 1);
    BufP out = alloc(1ull << lg);
    intt_nat(c, out->p, rot->p, lg, st);
    check_launch();
    self.b = out;
  }
  // Polynomial.divZh (polynomial.js:853-888): in place on the (possibly shared) buffer, then the
  // degree()+1 leading coefficients into a new buffer of 2^ceil(log2(deg + 1 - n)) (0 if deg < n)
  void div_zh(RPoly& self, uint64_t n) {
    const uint64_t ext = self.len() / n;
    const uint64_t deg0 = degree(self);
    const uint64_t length = deg0 < n ? 0 : 1ull << clog2(deg0 + 1 - n);
    HC(hipMemsetAsync(d_scratch + 1, 0, 4, st));
    self.b->written = true;
    launch_ref_divzh(st, self.b->p, n, (uint32_t)ext, d_scratch + 1);
    check_launch();
    HC(hipMemcpyAsync(h_scratch + 1, d_scratch + 1, 4, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    if (h_scratch[1]) throw KgsError(KGS_E_NOT_DIVISIBLE, "Polynomial is not divisible");
    const uint64_t d = degree(self);
    if (d + 1 > length) throw KgsError(KGS_E_RANGE, "offset is out of bounds");  // Q3
    RPoly q{zero(length)};
    HC(hipMemcpyAsync(q.b->p, self.b->p, 32 * (d + 1), hipMemcpyDeviceToDevice, st));
    self = q;
  }
};

}  // namespace

// The detection, enqueued on the main stream right after the quotient (no host round trip of its
// own: the caller reads the pinned block after its next sync): the degrees of the base operands
// (words 0..nops-1; length-n buffers), the degree of Q (word 8) and Q's coefficient 0 (words 16..23).
uint32_t* ref_quirks_probe(kgs_ctx& c, uint64_t n, const std::vector<const uint32_t*>& ops, const uint32_t* Q,
                           uint64_t qlen) {
  uint32_t* d = c.buf("refq_degs", 4 * 16);
  HC(hipMemsetAsync(d, 0, 4 * 16, c.st));
  for (size_t i = 0; i < ops.size() && i < 8; i++) launch_degree(c.st, d + i, ops[i], n);
  if (qlen) launch_degree(c.st, d + 8, Q, qlen);
  check_launch();
  uint32_t* h = (uint32_t*)c.pin(96);
  HC(hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, c.st));
  if (qlen) HC(hipMemcpyAsync(h + 16, Q, 32, hipMemcpyDeviceToHost, c.st));
  else memset(h + 16, 0, 32);
  return h;
}
// some base operand has a degree the reference's multiply mis-sizes (1 <= d < n/2)
bool ref_quirks_needed(const uint32_t* probe, size_t nops, uint64_t n) {
  for (size_t i = 0; i < nops && i < 8; i++)
    if (probe[i] >= 1 && 2ull * probe[i] < n) return true;
  return false;
}
// Q3 on the fast path: the dividend has degree < n iff the (exact) quotient is the zero polynomial
bool ref_quotient_is_zero(const uint32_t* probe) {
  if (probe[8]) return false;
  for (int j = 0; j < 8; j++)
    if (probe[16 + j]) return false;
  return true;
}

// The reference's quotient chain, op for op (prover.js:233-286 of either argument; `lookup` drops the
// selT-binary term). Inputs are the prover's own device buffers (coefficients, length n): polF / polT
// (the beta-combinations for vectors), S (or Z), selF / selT (nullptr: unselected). Throws what the
// reference throws ("Polynomial is not divisible", RangeError "offset is out of bounds"); otherwise
// returns the reference's Q (device buffer owned by the context pool, `qlen` = degree() + 1 of it, as
// multiExponentiation uses) and, when the chain wrote into polF's buffer (Q2, the unselected
// grand-sum's polQ1.add(polF) on a shorter polQ1), polF's values afterwards in `fmut` (else nullptr).
uint32_t* ref_quirks_quotient(kgs_ctx& c, bool gs, bool sel, bool lookup, int nbits, const Fr& alpha, const Fr& gamma,
                              const uint32_t* dF, const uint32_t* dT, const uint32_t* dS, const uint32_t* dSF,
                              const uint32_t* dST, uint64_t& qlen, uint32_t*& fmut) {
  const uint64_t n = 1ull << nbits;
  Engine E(c);
  RPoly polF = E.wrap(dF, n), polT = E.wrap(dT, n), polS = E.wrap(dS, n);
  const BufP polF_buf = polF.b, polT_buf = polT.b, polS_buf = polS.b;
  RPoly selF, selT;
  if (sel) {
    selF = E.wrap(dSF, n);
    selT = E.wrap(dST, n);
  }
  const BufP selF_buf = selF.b, selT_buf = selT.b;
  const Fr one = Fr::one();
  RPoly polQ = E.zero(n);  // prover.js:102
  if (sel) {
    if (!lookup) {
      RPoly b1 = E.clone(selT);
      E.multiply(b1, E.clone(selT));
      RPoly bin = E.clone(selT);
      E.sub(bin, b1);
      E.add(polQ, bin);
    }
    E.mul_scalar(polQ, alpha);
    RPoly b1 = E.clone(selF);
    E.multiply(b1, E.clone(selF));
    RPoly bin = E.clone(selF);
    E.sub(bin, b1);
    E.add(polQ, bin);
    E.mul_scalar(polQ, alpha);
  }
  RPoly polQ1 = E.clone(polS);
  E.shift_omega(polQ1);
  RPoly polFG = E.clone(polF);
  E.add_scalar(polFG, gamma);
  RPoly polTG = E.clone(polT);
  E.add_scalar(polTG, gamma);
  // Polynomial.Lagrange1 (polynomial.js:68-78): ifft of (1, 0, ..., 0) = every coefficient 1/n
  const Fr lag[2] = {one, Fr::from_u64(n).inverse()};
  const uint32_t* d_lag = c.scal(lag, 2);
  auto lagrange1 = [&]() {
    RPoly l{E.alloc(n)};
    launch_powers(E.st, l.b->p, n, d_lag, d_lag + 8);
    check_launch();
    return l;
  };
  if (gs) {  // src/grandsum/mset_eq_kzg_prover.js:252-282
    E.sub(polQ1, polS);
    E.multiply(polQ1, polFG);
    E.multiply(polQ1, polTG);
    if (sel) {
      RPoly sfg = E.clone(selF);
      E.multiply(sfg, polTG);
      RPoly stg = E.clone(selT);
      E.multiply(stg, polFG);
      E.add(polQ1, stg);
      E.sub(polQ1, sfg);
    } else {
      E.add(polQ1, polF);
      E.sub(polQ1, polT);
    }
    E.add(polQ, polQ1);
    E.mul_scalar(polQ, alpha);
    RPoly polQ2 = E.clone(polS);
    RPoly l1 = lagrange1();
    E.multiply(polQ2, l1);
    E.add(polQ, polQ2);
  } else {  // src/grandproduct/mset_eq_kzg_prover.js:252-282
    RPoly polQ2 = E.clone(polS);
    if (sel) {
      E.add_scalar(polTG, one.neg());
      E.multiply(polTG, E.clone(selT));
      E.add_scalar(polTG, one);
      E.multiply(polQ1, polTG);
      E.add_scalar(polFG, one.neg());
      E.multiply(polFG, E.clone(selF));
      E.add_scalar(polFG, one);
      E.multiply(polQ2, polFG);
    } else {
      E.multiply(polQ1, polTG);
      E.multiply(polQ2, polFG);
    }
    E.sub(polQ1, polQ2);
    E.add(polQ, polQ1);
    E.mul_scalar(polQ, alpha);
    RPoly polQ3 = E.clone(polS);
    E.add_scalar(polQ3, one.neg());
    RPoly l1 = lagrange1();
    E.multiply(polQ3, l1);
    E.add(polQ, polQ3);
  }
  E.div_zh(polQ, n);
  const uint64_t d = E.degree(polQ);
  qlen = polQ.len() ? d + 1 : 0;
  uint32_t* out = c.buf("refq_Q", 32 * (polQ.len() ? polQ.len() : 1));
  if (polQ.len()) HC(hipMemcpyAsync(out, polQ.b->p, 32 * polQ.len(), hipMemcpyDeviceToDevice, c.st));
  // Q2 can reach a base polynomial only through the unselected grand-sum's polQ1.add(polF) on a
  // shorter polQ1 (polF's buffer then holds polQ1 + F - T); rounds 4-5 read polF's buffer again
  fmut = nullptr;
  if (polF_buf->written) {
    fmut = c.buf("refq_Fmut", 32 * n);
    HC(hipMemcpyAsync(fmut, polF_buf->p, 32 * n, hipMemcpyDeviceToDevice, c.st));
  }
  for (const BufP* b : {&polT_buf, &polS_buf, &selF_buf, &selT_buf})
    if (*b && (*b)->written) throw KgsError(KGS_E_ARG, "reference-quirks mode: unexpected write into a shared base buffer");
  HC(hipStreamSynchronize(c.st));
  return out;
}

}  // namespace kgsi
