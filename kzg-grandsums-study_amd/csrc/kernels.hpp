// Launch wrappers for the gfx950 kernels (ntt.hip, poly.hip, msm.hip). All pointers are device
// pointers to 32 B Montgomery Fr elements (uint32_t[8]) or 64 B affine / 128 B XYZZ G1 points,
// unless stated otherwise. Launches are asynchronous on `st`.
#pragma once

// Wave priority: every kernel except k_accumulate raises its waves to priority 3 (1 until round 5), so the
// short latency-bound kernels of the other in-flight proofs (NTT, sort, MSM tail, poly) win VALU arbitration
// against the long accumulate waves they share SIMDs with (arbitration is by priority, then age); the
// accumulate waves stay at 0, or step 2 -> 1 -> 0 with their progress (msm.hip, k_accumulate). A/B on
// MI355X, same box: 77.9 -> 80.5 proofs/s at n = 2^20 (4 in flight); single-proof latency 14.6 -> 14.9 ms.
// -DKGS_NO_PRIO_AUX disables.
#ifndef KGS_NO_PRIO_AUX
#define KGS_AUX_PRIO() __builtin_amdgcn_s_setprio(3)
#else
#define KGS_AUX_PRIO() ((void)0)
#endif

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "field.hpp"

namespace kgs {

constexpr int LC_MAX = 32;
constexpr int LC_W29 = 10;  // words of a coefficient's 29-bit product record (fr29.hpp)
struct LinComb {  // out[i] = sum_k coef_k * src_k[i] (zero beyond len_k) + (i == 0 ? c0 : 0)
  int nterms;
  const uint32_t* src[LC_MAX];
  uint64_t len[LC_MAX];
  uint32_t coef[LC_MAX][8];
  uint32_t coef29[LC_MAX][LC_W29];  // coef_k as 29-bit records (prover.cpp fr29_record)
  uint32_t c0[8];
};

constexpr int EB_MAX = 32;
struct EvalBatch {
  int npolys;
  const uint32_t* src[EB_MAX];
  uint64_t len[EB_MAX];
};

struct MsmTables {
  uint32_t* table = nullptr;  // W x npts affine points (64 B)
  uint64_t npts = 0;
  int c = 0, W = 0;
};

constexpr int MSM_SL_G_MAX = 128;  // chunks per partition the lo-pass count buffer holds (msm.hip SL_G)
// Bucket sort of an MSM with window c (msm.hip): LOB low bits of key - 1 are sorted inside a partition
// (<= 8: the lo pass keeps them in a byte), the other c - 1 - LOB bits select one of NH = 2^(c-1-LOB)
// partitions: 256 for 16 <= c <= 17, 512 / 1024 / 2048 for c = 18 / 19 / 20
constexpr int MSM_NH_MAX = 2048;
inline int msm_lob(int c) {
  int lob = c - 1 < 7 ? c - 1 : 7;
  if (c - 9 > lob) lob = c - 9 > 8 ? 8 : c - 9;
  return lob;
}
inline int msm_nh(int c) { return (1 << (c - 1)) >> msm_lob(c); }
struct MsmWork {
  int32_t* digit = nullptr;  // reused as the partition-pass value array
  uint8_t* lo = nullptr;
  uint32_t* blockhist = nullptr;  // NH x ceil(N / (256 * SORT_SPT)) per-block partition counts
  uint32_t *counts = nullptr, *offsets = nullptr, *cursor = nullptr, *sorted = nullptr;
  uint32_t* part = nullptr;      // bucket row + column sums (2^h + 2^l run records, msm.hip k_rowcol)
  uint32_t* segowner = nullptr;  // bucket of each segment's first run
  uint32_t* locnt = nullptr;     // lo pass: NH partitions x 256 lo x MSM_SL_G_MAX chunks counts / bases
  uint32_t* chunklist = nullptr; // combine levels: 3 lists of chunk-start segments
  uint32_t* chunkcnt = nullptr;  // their lengths
  uint32_t* raw29 = nullptr;     // accumulate output in the fq29 form (B + 1 + nseg entries x 160 B)
};

// ntt.hip
// NTT LDS passes built for three waves per SIMD (co-resident with two accumulate waves: proofs in
// flight) or two (fastest alone) for the calling thread's later launches; returns the previous setting
bool ntt_set_coresident(bool on);
constexpr int TW29_WORDS = 10;  // words per 29-bit twiddle record (fr29.hpp W29_WORDS)
// the 29-bit twin (fr29.hpp, k_tw29 records; record i <-> element i) of `count` 8 x 32 elements at
// `base`: the LDS passes of ntt_dif / ntt_dit multiply by the twin records of the twiddle table and
// the pre / post scalings they were given when every one of them lies in a registered table
void ntt_register_tw29(const uint32_t* base, uint64_t count, const uint32_t* twin);
void ntt_unregister_tw29(const uint32_t* base);
// out[i] = the k_tw29 record of in[i] (8 x 32 Montgomery words), i < count
void launch_tw29(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t count);
void ntt_dif(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t in_len, int logm, const uint32_t* pre,
             const uint32_t* tw, int logM);
void ntt_dit(hipStream_t st, uint32_t* out, const uint32_t* in, int in_bitrev, int logm, const uint32_t* tw, int logM,
             const uint32_t* post, const uint32_t* post_s);
void launch_powers(hipStream_t st, uint32_t* out, uint64_t count, const uint32_t* w_dev, const uint32_t* scale_dev);
void launch_scale_copy(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n, const uint32_t* tab,
                       const uint32_t* sc);
void launch_bitrev_copy(hipStream_t st, uint32_t* out, const uint32_t* in, int logm);

// poly.hip
void launch_to_mont(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n);
// device -> mapped pinned host memory by a small store kernel (bytes a multiple of 16)
void launch_host_store(hipStream_t st, void* dst_host_mapped, const void* src, uint64_t bytes, unsigned blocks);
void launch_lincomb(hipStream_t st, uint32_t* out, uint64_t n, const LinComb& lc);
void launch_builder(hipStream_t st, bool prod, bool sel, uint32_t* out, const uint32_t* f, const uint32_t* t,
                    const uint32_t* sf, const uint32_t* stt, const uint32_t* gamma, uint64_t n, uint32_t* scratch_tp,
                    uint32_t* scratch_ti, uint32_t* flag);
void launch_quotient(hipStream_t st, bool prod, bool sel, uint32_t* q, const uint32_t* S, const uint32_t* F,
                     const uint32_t* T, const uint32_t* SF, const uint32_t* ST, const uint32_t* inv_nxm1,
                     const uint32_t* scalars, int lcs, uint32_t rot);
void launch_divcheck(hipStream_t st, bool prod, bool sel, uint32_t* flag, const uint32_t* S, const uint32_t* f,
                     const uint32_t* t, const uint32_t* sf, const uint32_t* stt, const uint32_t* scalars, uint64_t n,
                     const uint32_t* S_next = nullptr, uint64_t gbase = 0);
void launch_eval_tiles(hipStream_t st, uint32_t* part, const EvalBatch& eb, const uint32_t* xp, uint32_t ntiles_max);
void launch_divide(hipStream_t st, uint32_t* q, uint32_t* flag, const uint32_t* a, uint64_t L, const uint32_t* xp,
                   uint32_t* part, uint32_t* carry);
void launch_fr_batch_inv(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n);
void launch_from_mont(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n);
void launch_nxm1(hipStream_t st, uint32_t* out, const uint32_t* tw, uint64_t halfM, const uint32_t* gp,
                 const uint32_t* np, int lcs, uint64_t wstride);
constexpr uint64_t EVAL_TILE = 2048;
// reference-quirks mode (prover.cpp ref_quirks_*): degree, the reference's multiply/shiftOmega
// pointwise step on its own evaluation domains, divZh in place
void launch_degree(hipStream_t st, uint32_t* out, const uint32_t* a, uint64_t len);
void launch_ref_gather_mul(hipStream_t st, uint32_t* out, const uint32_t* a, int loga, const uint32_t* b, int logb,
                           uint64_t N, uint64_t rot);
void launch_ref_divzh(hipStream_t st, uint32_t* c, uint64_t n, uint32_t ext, uint32_t* flag);

// dist.hip (the distributed prover's rank-local kernels; layouts in prover_dist.cpp)
void launch_gather_e(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t N, int W, int r, bool to_mont);
void launch_dfwd_pack(hipStream_t st, uint32_t* send, const uint32_t* Z, int logMl, int W, int r, const uint32_t* tw,
                      int logN);
void launch_dfwd_wdft(hipStream_t st, uint32_t* out, const uint32_t* recv, int logMl, int W, const uint32_t* tw, int logN);
void launch_dinv_wdft_pack(hipStream_t st, uint32_t* send, const uint32_t* loc, int logMl, int W, int r,
                           const uint32_t* tw_inv, int logN);
void launch_unpack_c2b(hipStream_t st, uint32_t* out, const uint32_t* recv, uint64_t Lb, int W);
void launch_pack_b2c(hipStream_t st, uint32_t* send, const uint32_t* blk, uint64_t Lb, int W);
void launch_scan_fix(hipStream_t st, bool prod, uint32_t* out, const uint32_t* off, uint64_t n);
void launch_e_heads(hipStream_t st, uint32_t* heads, const uint32_t* S, uint64_t Ml, int W, int rot);
void launch_quotient_e(hipStream_t st, bool prod, bool sel, uint32_t* q, const uint32_t* S, const uint32_t* F,
                       const uint32_t* T, const uint32_t* SF, const uint32_t* ST, const uint32_t* nxm1,
                       const uint32_t* scalars, const uint32_t* halo, uint64_t Ml, int W, int r, int rot);
void launch_nxm1_e(hipStream_t st, uint32_t* out, const uint32_t* tw, int lcs, const uint32_t* gp, const uint32_t* np,
                   int W, int r);
void launch_div_fix(hipStream_t st, uint32_t* q, const uint32_t* pz, const uint32_t* c, uint64_t Lb);

// msm.hip
void msm_build_table(hipStream_t st, uint32_t* table, uint64_t npts, int c, int W, uint32_t* tmp_xyzz,
                     uint32_t* scratch);
// scalars[i] multiplies SRS point pbase + pstride * i (pbase + pstride * (N - 1) < tb.npts).
// exclusive_acc: the bucket accumulation takes a SIMD's whole register file at its two waves (for a
// context whose two MSM lanes would otherwise co-run their accumulations and delay each other's
// tails); default: a 168-VGPR build that leaves room for other proofs' kernels (msm.hip).
void msm_run(hipStream_t st, const MsmTables& tb, MsmWork& w, const uint32_t* scalars, uint64_t N, uint32_t* T_out,
             hipEvent_t* ev = nullptr, uint64_t pbase = 0, uint64_t pstride = 1, bool exclusive_acc = false);
void launch_fixed_base(hipStream_t st, uint32_t* out_xyzz, const uint32_t* sc, uint64_t count, const uint32_t* tbl);
void launch_batch_affine(hipStream_t st, uint32_t* out_aff, const uint32_t* in_xyzz, uint32_t* scratch, uint64_t npts);

}  // namespace kgs
