// Native verifiers for both arguments (host C++, no GPU): kgs_verify / kgs_verify_ptau.
//
// Restates src/grandsum/mset_eq_kzg_verifier.js:9-313 and
// src/grandproduct/mset_eq_kzg_verifier.js:9-299 step by step: validate the commitments (on G1)
// and the evaluations (< r), replay the Keccak transcript (beta only for vector arguments; an
// absent beta multiplies zero, Appendix C.4 of SURVEY.md), evaluate Z_H(xi) and L1(xi), build
// r0, [D]1, [F]1, [E]1, and decide e(-A, [tau]2) * e(B, [1]2) == 1 with the optimal-ate pairing.
// Inputs use the fixed C-ABI order of kgs_prove (include/kgs.h, kgs_proof_shape).
#include <stdio.h>
#include <string.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/kgs.h"
#include "host_field.hpp"
#include "host_pairing.hpp"
#include "transcript.hpp"

using namespace kgs;
using host::Fq;
using host::Fr;
using host::G1;

namespace {

bool lt_mod(const uint8_t* le, const uint64_t* p) {  // little-endian 256-bit value < p
  for (int i = 3; i >= 0; i--) {
    uint64_t w;
    memcpy(&w, le + 8 * i, 8);
    if (w != p[i]) return w < p[i];
  }
  return false;
}

// G1.isValid on an affine LEM point: infinity, or canonical coordinates on y^2 = x^3 + 3
bool g1_valid(const uint8_t* lem) {
  bool zero = true;
  for (int i = 0; i < 64; i++) zero &= lem[i] == 0;
  if (zero) return true;
  if (!lt_mod(lem, host::FQ_MOD.p) || !lt_mod(lem + 32, host::FQ_MOD.p)) return false;
  Fq x = Fq::from_bytes(lem), y = Fq::from_bytes(lem + 32);
  return y.sqr() == x.sqr() * x + Fq::from_u64(3);
}

struct Proof {
  int npols;
  bool sel, gs;
  const uint8_t* com;  // fixed order (kgs_proof_shape)
  const uint8_t* ev;
  bool lookup = false;  // KGS_LOOKUP: no binary constraint on selT
  // commitment indices
  const uint8_t* F(int i) const { return com + 64 * (2 * i); }
  const uint8_t* T(int i) const { return com + 64 * (2 * i + 1); }
  const uint8_t* selF() const { return com + 64 * (2 * npols); }
  const uint8_t* selT() const { return com + 64 * (2 * npols + 1); }
  int base() const { return 2 * npols + (sel ? 2 : 0); }
  const uint8_t* S() const { return com + 64 * base(); }  // S (grand-sum) or Z (grand-product)
  const uint8_t* Q() const { return com + 64 * (base() + 1); }
  const uint8_t* Wxi() const { return com + 64 * (base() + 2); }
  const uint8_t* Wxiw() const { return com + 64 * (base() + 3); }
  int ncom() const { return base() + 4; }
  // evaluation indices: per pol f (and t for grand-sum), then selF, selT, then S(xi w) / Z(xi w)
  int per() const { return gs ? 2 : 1; }
  const uint8_t* fxi_raw(int i) const { return ev + 32 * (per() * i); }
  const uint8_t* txi_raw(int i) const { return ev + 32 * (per() * i + 1); }
  const uint8_t* selFxi_raw() const { return ev + 32 * (per() * npols); }
  const uint8_t* selTxi_raw() const { return ev + 32 * (per() * npols + 1); }
  const uint8_t* sxiw_raw() const { return ev + 32 * (per() * npols + (sel ? 2 : 0)); }
  int nev() const { return per() * npols + (sel ? 2 : 0) + 1; }
};

Fr fr_at(const uint8_t* b) { return Fr::from_bytes(b); }
G1 pt(const uint8_t* lem) { return G1::from_affine_lem(lem); }

bool verify_impl(const Proof& p, int nbits, const host::G2A& tau_g2) {
  const int k = p.npols;
  const bool vec = k > 1;
  // validateCommitments / validateEvaluations (grandsum verifier.js:194-244, grandproduct :200-233)
  for (int i = 0; i < p.ncom(); i++)
    if (!g1_valid(p.com + 64 * i)) return false;
  for (int i = 0; i < p.nev(); i++)
    if (!lt_mod(p.ev + 32 * i, host::FR_MOD.p)) return false;

  // computeChallenges (grandsum verifier.js:246-312)
  host::Transcript tr;
  for (int i = 0; i < k; i++) {
    tr.add_commitment(p.F(i));
    tr.add_commitment(p.T(i));
  }
  if (p.sel) {
    tr.add_commitment(p.selF());
    tr.add_commitment(p.selT());
  }
  Fr beta = Fr::zero();
  if (vec) {
    beta = tr.challenge();
    tr.add_scalar(beta);
  }
  const Fr gamma = tr.challenge();
  tr.add_scalar(gamma);
  tr.add_commitment(p.S());
  const Fr alpha = tr.challenge();
  tr.add_scalar(alpha);
  tr.add_commitment(p.Q());
  const Fr xi = tr.challenge();
  tr.add_scalar(xi);
  for (int i = 0; i < k; i++) {
    tr.add_scalar(fr_at(p.fxi_raw(i)));
    if (p.gs) tr.add_scalar(fr_at(p.txi_raw(i)));
  }
  if (p.sel) {
    tr.add_scalar(fr_at(p.selFxi_raw()));
    tr.add_scalar(fr_at(p.selTxi_raw()));
  }
  const Fr sxiw = fr_at(p.sxiw_raw());
  tr.add_scalar(sxiw);
  const Fr v = tr.challenge();
  tr.add_scalar(v);
  tr.add_commitment(p.Wxi());
  tr.add_commitment(p.Wxiw());
  const Fr u = tr.challenge();

  // Z_H(xi), L1(xi) (polynomial_utils.js:1-19)
  Fr xn = xi;
  for (int i = 0; i < nbits; i++) xn = xn.sqr();
  const Fr zh = xn - Fr::one();
  const Fr l1 = zh * (Fr::from_u64(1ull << nbits) * (xi - Fr::one())).inverse();
  const Fr w = host::fr_w(nbits);

  Fr r0 = Fr::zero();
  Fr selF = Fr::zero(), selT = Fr::zero();
  if (p.sel) {
    selF = fr_at(p.selFxi_raw());
    selT = fr_at(p.selTxi_raw());
    if (!p.lookup) r0 = r0 + (selT - selT.sqr());  // a lookup's selT holds multiplicities
    r0 = r0 * alpha;
    r0 = (r0 + (selF - selF.sqr())) * alpha;
  }
  Fr fxi = Fr::zero(), txi = Fr::zero();
  for (int i = k - 1; i >= 0; i--) {
    fxi = fxi * beta + fr_at(p.fxi_raw(i));
    if (p.gs) txi = txi * beta + fr_at(p.txi_raw(i));
  }
  G1 D1;
  if (p.gs) {
    const Fr fg = fxi + gamma, tg = txi + gamma;
    Fr r01 = sxiw * (fg * tg);
    if (p.sel)
      r01 = r01 + selT * fg - selF * tg;
    else
      r01 = r01 + fxi - txi;
    r0 = (r0 + r01) * alpha;
    const Fr d11 = (l1 - alpha * fg * tg) + u;
    D1 = pt(p.S()).mul(d11).add(pt(p.Q()).mul(zh).neg());
  } else {
    Fr r01 = sxiw;
    r01 = p.sel ? r01 * ((gamma - Fr::one()) * selT + Fr::one()) : r01 * gamma;
    r0 = (r0 + r01) * alpha;
    r0 = r0 - l1;
    Fr fg = fxi + gamma;
    if (p.sel) fg = (fg - Fr::one()) * selF + Fr::one();
    const Fr d11 = (l1 - alpha * fg) + u;
    G1 D12 = G1::inf();
    for (int i = k - 1; i >= 0; i--) D12 = D12.mul(beta).add(pt(p.T(i)));
    if (p.sel) D12 = D12.mul(selT);
    D12 = D12.mul(sxiw).mul(alpha);
    D1 = pt(p.S()).mul(d11).add(D12).add(pt(p.Q()).mul(zh).neg());
  }
  // [F]1 (grandsum verifier.js:125-142)
  G1 F1 = G1::inf();
  if (p.sel) {
    F1 = F1.add(pt(p.selT()));
    F1 = F1.mul(v).add(pt(p.selF()));
  }
  if (p.gs)
    for (int i = k - 1; i >= 0; i--) F1 = F1.mul(v).add(pt(p.T(i)));
  for (int i = k - 1; i >= 0; i--) F1 = F1.mul(v).add(pt(p.F(i)));
  F1 = F1.mul(v).add(D1);
  // [E]1 (:146-167)
  Fr E = Fr::zero();
  if (p.sel) {
    E = E + selT;
    E = E * v + selF;
  }
  if (p.gs)
    for (int i = k - 1; i >= 0; i--) E = E * v + fr_at(p.txi_raw(i));
  for (int i = k - 1; i >= 0; i--) E = E * v + fr_at(p.fxi_raw(i));
  E = E * v + u * sxiw - r0;
  uint8_t g1gen[64];
  Fq::one().to_bytes(g1gen);
  Fq::from_u64(2).to_bytes(g1gen + 32);
  const G1 E1 = pt(g1gen).mul(E);
  // pairing equation (:170-186)
  const G1 A = pt(p.Wxi()).add(pt(p.Wxiw()).mul(u));
  G1 Bp;
  if (p.gs)
    Bp = pt(p.Wxi()).add(pt(p.Wxiw()).mul(u * w)).mul(xi);
  else
    Bp = pt(p.Wxi()).mul(xi).add(pt(p.Wxiw()).mul(u * xi * w));
  Bp = Bp.add(F1).add(E1.neg());
  return host::pairing_eq2(A.neg(), tau_g2, Bp, host::g2_gen());
}

thread_local std::string v_err;

}  // namespace

extern "C" {

int kgs_proof_shape(int kind, int npols, int selected, int* n_commitments, int* n_evaluations) {
  if (npols < 1 || npols > (1 << 20)) return KGS_E_ARG;
  if (n_commitments) *n_commitments = 2 * npols + (selected ? 2 : 0) + 4;
  if (kind != KGS_GRANDSUM && kind != KGS_GRANDPRODUCT && kind != KGS_LOOKUP) return KGS_E_ARG;
  if (n_evaluations) *n_evaluations = (kind != KGS_GRANDPRODUCT ? 2 : 1) * npols + (selected ? 2 : 0) + 1;
  return KGS_OK;
}

int kgs_verify(int kind, int nbits, int npols, int selected, const uint8_t* commitments, const uint8_t* evaluations,
               const uint8_t tau_g2[128]) {
  if ((kind != KGS_GRANDSUM && kind != KGS_GRANDPRODUCT && kind != KGS_LOOKUP) || (kind == KGS_LOOKUP && !selected) ||
      nbits < 1 || nbits > 28 || npols < 1 || !commitments ||
      !evaluations || !tau_g2)
    return KGS_E_ARG;
  try {
    Proof p{npols, selected != 0, kind != KGS_GRANDPRODUCT, commitments, evaluations, kind == KGS_LOOKUP};
    host::G2A t2 = host::g2_from_lem(tau_g2);
    if (!host::g2_on_curve(t2)) return KGS_E_ARG;
    return verify_impl(p, nbits, t2) ? 1 : 0;
  } catch (const std::exception&) {
    return KGS_E_ARG;
  }
}

int kgs_pairing_eq(int npairs, const uint8_t* g1_lem, const uint8_t* g2_lem) {
  if (npairs < 0 || npairs > 4096 || (npairs && (!g1_lem || !g2_lem))) return KGS_E_ARG;
  try {
    std::vector<host::G1> a(npairs);
    std::vector<host::G2A> b(npairs);
    std::vector<const host::G1*> pa(npairs);
    std::vector<const host::G2A*> pb(npairs);
    for (int k = 0; k < npairs; k++) {
      const uint8_t* p1 = g1_lem + 64 * (size_t)k;
      if (!host::g1_lem_on_curve(p1)) return KGS_E_ARG;
      a[k] = host::G1::from_affine_lem(p1);
      b[k] = host::g2_from_lem(g2_lem + 128 * (size_t)k);
      if (!host::g2_on_curve(b[k])) return KGS_E_ARG;
      pa[k] = &a[k];
      pb[k] = &b[k];
    }
    return host::pairing_eq(pa.data(), pb.data(), npairs) ? 1 : 0;
  } catch (const std::exception&) {
    return KGS_E_ARG;
  }
}

int kgs_verify_ptau(int kind, const char* ptau_path, int nbits, int npols, int selected, const uint8_t* commitments,
                    const uint8_t* evaluations) {
  uint8_t t2[128];
  int rc = kgs_ptau_read_tau_g2(ptau_path, t2);
  if (rc < 0) return rc;
  return kgs_verify(kind, nbits, npols, selected, commitments, evaluations, t2);
}

}  // extern "C"
