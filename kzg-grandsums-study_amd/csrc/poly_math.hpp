// Per-point arithmetic of the quotient numerator, shared by the single-GPU kernels (poly.hip) and
// the distributed ones (dist.hip) so that both compute identical values.
// Grand-sum (prover.js:233-286):
//   N(x) = alpha [ (S(wx) - S(x)) (F+g)(T+g) + (T+g) selF - (F+g) selT ]  (unselected: + F - T)
//          + alpha^2 (selF - selF^2) + alpha^3 (selT - selT^2)  + L1(x) S(x)
// The selT-binary term is weighted by alpha_t = alpha (grand-sum) or 0 (KGS_LOOKUP: selT carries
// multiplicities), so both arguments share one kernel and the grand-sum values are unchanged.
// Grand-product (grandproduct prover.js:233-286): alpha [ Z(wx) dT - Z(x) dF ] + ... + L1(x) (Z(x) - 1)
#pragma once
#include "field.hpp"

namespace kgs {

// sel terms + main term, before the outer factor alpha (k_quotient folds alpha into 1/Z_H)
template <bool PROD, bool SEL>
__device__ __forceinline__ fr quotient_core_na(const fr& s, const fr& sw, const fr& fv, const fr& tv, const fr& sf,
                                               const fr& st, const fr& alpha, const fr& gamma,
                                               const fr& alpha_t) {
  const fr fg = fv + gamma, tg = tv + gamma;
  fr acc = fr::zero();
  if (SEL) {
    // alpha^3 (selT - selT^2) + alpha^2 (selF - selF^2)  ==  ((selT-selT^2)*alpha + (selF-selF^2))*alpha^2
    acc = (st - st.sqr()) * alpha_t + (sf - sf.sqr());
    acc = acc * alpha;  // multiplied by alpha once more below together with the main term
  }
  fr q1;
  if (!PROD) {
    q1 = (sw - s) * fg * tg;
    if (SEL) q1 = q1 + st * fg - sf * tg;
    else q1 = q1 + (fg - tg);  // F - T
  } else {
    const fr one = fr::one();
    fr dT = tg, dF = fg;
    if (SEL) {
      dT = st * (tg - one) + one;
      dF = sf * (fg - one) + one;
    }
    q1 = sw * dT - s * dF;
  }
  return acc + q1;
}
// alpha * (sel terms + main term); L1 part added by the caller
template <bool PROD, bool SEL>
__device__ __forceinline__ fr quotient_core(const fr& s, const fr& sw, const fr& fv, const fr& tv, const fr& sf,
                                            const fr& st, const fr& alpha, const fr& gamma,
                                            const fr& alpha_t) {
  return quotient_core_na<PROD, SEL>(s, sw, fv, tv, sf, st, alpha, gamma, alpha_t) * alpha;
}

// L1(x) S(x) / Z_H(x) with L1/Z_H = 1/(n(x - 1)) = nxm1; grand-product uses Z(x) - 1
template <bool PROD>
__device__ __forceinline__ fr quotient_l1(const fr& s, const fr& nxm1) {
  return (PROD ? s - fr::one() : s) * nxm1;
}

}  // namespace kgs
