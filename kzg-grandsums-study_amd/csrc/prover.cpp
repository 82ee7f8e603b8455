// Host orchestration of the MI355X-native grand-sum / grand-product KZG prover + the C-ABI
// (include/kgs.h). One context = one device, one HIP stream, a device-resident SRS with its MSM
// window tables, NTT/coset tables, and a grow-only device buffer pool.
//
// Round structure, transcript order and proof schema follow the reference provers exactly
// (src/grandsum/mset_eq_kzg_prover.js:12-434, src/grandproduct/mset_eq_kzg_prover.js:12-414).
// Every output is a unique field / group element, so the computation is re-planned for the GPU
// where that leaves the values unchanged (DESIGN.md §Hot path):
//  * evalsF = fft(sum beta^i F_i) = sum beta^i f_i (NTT linearity; prover.js:207-217)
//  * the quotient Q = N / Z_H is computed on a coset of size 2n (n for the unselected grand
//    product) instead of the 2n/4n `multiply` chain + `divZh` (prover.js:233-286); divisibility
//    (the "Polynomial is not divisible" check of divZh) is decided exactly by N(w^i) == 0 on H;
//  * S(wX) on the coset is a rotation of the coset evaluations (no shiftOmega NTT pair);
//  * L1(X)/Z_H(X) = 1/(n (X - 1)) on the coset (precomputed per domain);
//  * commitments skip zero top coefficients by degree bounds (zero scalars add nothing).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <algorithm>
#include <map>
#include <mutex>
#include <sys/stat.h>
#include <memory>
#include <stdexcept>
#include <string>
#include <functional>
#include <atomic>
#include <thread>
#include <immintrin.h>
#include <vector>

#include "../../include/kgs.h"
#include "host_field.hpp"
#include "host_pairing.hpp"
#include "kernels.hpp"
#include "host_error.hpp"
#ifndef KGS_NO_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif
#include "keccak.hpp"
#include "ptau_io.hpp"
#include "transcript.hpp"

#include <condition_variable>
#include "context.hpp"

using namespace kgs;
using namespace kgsi;
using host::Fq;
using host::Fr;

namespace kgsi {

// Every device allocation goes through here. KGS_DEBUG_ALLOC_LIMIT=<bytes> (fault injection for the
// tests) makes any single request above that size fail as out-of-memory; with KGS_DEBUG_ALLOC_RANK=<r>
// only on the host thread that is proving as rank r of a rank group (a failure on ONE rank of an
// in-process group, whose ranks are threads of one process).
thread_local int tl_group_rank = -1;
hipError_t dev_malloc(void** p, size_t bytes) {
  if (const char* e = getenv("KGS_DEBUG_ALLOC_LIMIT")) {
    const unsigned long long lim = strtoull(e, nullptr, 10);
    const char* rk = getenv("KGS_DEBUG_ALLOC_RANK");
    if (lim && bytes > lim && (!rk || atoi(rk) == tl_group_rank)) {
      *p = nullptr;
      return hipErrorOutOfMemory;
    }
  }
  return hipMalloc(p, bytes);
}

std::mutex g_reg_mu;
std::vector<std::weak_ptr<SrsTables>> g_srs_reg;
std::vector<std::weak_ptr<DomainTables>> g_dom_reg;

}  // namespace kgsi

namespace kgsi {

// ------------------------------------------------------------------ domain tables
// The 29-bit twin of every table (stage twiddles, coset powers, 1/m), record i <-> element i, for the
// LDS passes' products (fr29.hpp): 40 B per element beside the 32 B words. Built with the domain for
// the proofs' own domains; a domain grown only for the reference-quirks replay (up to 2^26 points)
// gets none (its NTTs take the 8 x 32 products, the same values), and the first proof that runs on it
// builds the twin then (ensure_twin). Under g_reg_mu.
static void build_twin(kgs_ctx& c, DomainTables* d) {
  if (d->mem29) return;
  const uint64_t entries = 4 * (1ull << d->logM) + d->logM + 1;
  HC(dev_malloc((void**)&d->mem29, (size_t)4 * TW29_WORDS * entries));
  launch_tw29(c.st, d->mem29, d->mem, entries);
  check_launch();
  HC(hipStreamSynchronize(c.st));
  ntt_register_tw29(d->mem, entries, d->mem29);
}
void ensure_twin(kgs_ctx& c) {
  if (!c.dom) return;
  std::lock_guard<std::mutex> lk(g_reg_mu);  // mem29 is written under this lock (by any context)
  build_twin(c, c.dom.get());
}

// Shared per device: a context asking for 2^logM reuses any published table of at least that size.
void ensure_domain(kgs_ctx& c, int logM, bool twin) {
  if (c.logM >= logM) return;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (auto& w : g_dom_reg) {
    auto d = w.lock();
    if (d && d->device == c.device && d->logM >= logM) {
      if (twin) build_twin(c, d.get());
      // switching may drop the last reference to the old tables (freed at once): nothing of this
      // context may still read them. Every caller drains its streams first today; this keeps it so.
      c.sync();
      c.use_domain(d);
      c.nxm1.clear();
      return;
    }
  }
  const uint64_t M = 1ull << logM;
  auto d = std::make_shared<DomainTables>();
  d->device = c.device;
  // stage twiddle tables: tw[h + t] = w_{2h}^t for h = 2^l, l < logM (entries 1..M-1); coset powers
  // g^i, g^-i (g = 5); 1/2^l for l <= logM
  const size_t words = (size_t)8 * (4 * M + logM + 1);
  HC(dev_malloc((void**)&d->mem, 4 * words));
  d->tw_fwd = d->mem;
  d->tw_inv = d->tw_fwd + 8 * M;
  d->coset_pow = d->tw_inv + 8 * M;
  d->coset_ipow = d->coset_pow + 8 * M;
  d->invm = d->coset_ipow + 8 * M;
  // This may run in the middle of a proof (the reference-quirks replay grows the domain,
  // ref_quirks.cpp need_domain): the scalars and pinned words the proof has staged so far must stay
  // intact, so the build stages above them and gives that space back once it has completed.
  c.sync();
  const size_t pin_mark = c.h_pin_off, scal_mark = c.d_scal_off;
  std::vector<Fr> consts;
  for (int l = 0; l < logM; l++) {
    Fr w = fr_w(l + 1);
    consts.push_back(w);
    consts.push_back(w.inverse());
  }
  Fr g = Fr::from_u64(5);
  consts.push_back(g);
  consts.push_back(g.inverse());
  uint32_t* dc = c.scal(consts.data(), (int)consts.size());
  for (int l = 0; l < logM; l++) {
    const uint64_t h = 1ull << l;
    launch_powers(c.st, d->tw_fwd + 8 * h, h, dc + 16 * l, nullptr);
    launch_powers(c.st, d->tw_inv + 8 * h, h, dc + 16 * l + 8, nullptr);
  }
  launch_powers(c.st, d->coset_pow, M, dc + 16 * logM, nullptr);
  launch_powers(c.st, d->coset_ipow, M, dc + 16 * logM + 8, nullptr);
  std::vector<Fr> im(logM + 1);
  for (int l = 0; l <= logM; l++) im[l] = Fr::from_u64(1ull << l).inverse();
  uint8_t* h = c.pin(32 * (logM + 1));
  for (int l = 0; l <= logM; l++) im[l].to_bytes(h + 32 * l);
  HC(hipMemcpyAsync(d->invm, h, 32 * (logM + 1), hipMemcpyHostToDevice, c.st));
  check_launch();
  c.sync();  // built
  c.h_pin_off = pin_mark;
  c.d_scal_off = scal_mark;
  d->logM = logM;
  if (twin) build_twin(c, d.get());  // then publish
  g_dom_reg.erase(std::remove_if(g_dom_reg.begin(), g_dom_reg.end(), [](auto& w) { return w.expired(); }),
                  g_dom_reg.end());
  g_dom_reg.push_back(d);
  c.use_domain(d);
  c.nxm1.clear();
}

uint32_t* get_nxm1(kgs_ctx& c, int nbits, int lcs) {
  auto key = std::make_pair(nbits, lcs);
  auto it = c.nxm1.find(key);
  if (it != c.nxm1.end()) return it->second;
  const uint64_t cs = 1ull << lcs;
  uint32_t* out = c.buf("nxm1_" + std::to_string(nbits) + "_" + std::to_string(lcs), 32 * cs);
  uint32_t* tmp = c.buf("nxm1_tmp", 32 * cs);
  // 1/(n (x - 1)) / cs: the coset inverse NTT of the quotient (coset_inv_prescaled) takes its 1/cs from here and
  // from the Z_H scalars of round 3 instead of a product per element
  Fr consts[2] = {Fr::from_u64(5), Fr::from_u64(1ull << nbits) * Fr::from_u64(cs)};
  uint32_t* d = c.scal(consts, 2);
  // w_M^j (j < M/2) is the last stage table, tw_fwd + 8 * (M/2)
  const uint64_t halfM = (1ull << c.logM) / 2;
  launch_nxm1(c.st, tmp, c.tw_fwd + 8 * halfM, halfM, d, d + 8, lcs, (1ull << c.logM) >> lcs);
  launch_fr_batch_inv(c.st, out, tmp, cs);
  check_launch();
  c.nxm1[key] = out;
  return out;
}

// ------------------------------------------------------------------ NTT helpers
// natural-order evaluations -> natural-order coefficients (out != in)
void intt_nat(kgs_ctx& c, uint32_t* out, const uint32_t* in, int logm, hipStream_t st) {
  ntt_dit(st ? st : c.st, out, in, 0, logm, c.tw_inv, c.logM, nullptr, c.invm + 8 * logm);
}
// coefficients (len <= 2^lcs, natural) -> coset evaluations p(g w^i), bit-reversed order
void coset_fwd(kgs_ctx& c, uint32_t* out, const uint32_t* in, uint64_t len, int lcs, hipStream_t st) {
  ntt_dif(st ? st : c.st, out, in, len, lcs, c.coset_pow, c.tw_fwd, c.logM);
}
// bit-reversed coset evaluations, already scaled by 1/cs -> natural coefficients (in place allowed)
void coset_inv_prescaled(kgs_ctx& c, uint32_t* out, const uint32_t* in, int lcs) {
  ntt_dit(c.st, out, in, 1, lcs, c.tw_inv, c.logM, c.coset_ipow, nullptr);
}

// ------------------------------------------------------------------ SRS
// Window c of the MSM tables of `npts` resident points: lg - 4, between 7 and 17. The bucket entries
// of an N-point MSM are N * ceil(255 / c) XYZZ mixed adds, its bucket tail (row / column sums) ~2^c
// full adds. Windows up to c = 20 are built and parity-tested (KGS_MSM_C, the sort's partitions grow
// to 2048), but c = 20 at n = 2^20 measured slower: 13 windows instead of 15 cut the accumulation
// 1.25 -> 1.10 ms, while the sort went 0.15 -> 0.30 ms and the tail 0.21 -> 0.53 ms, 93.3 -> 85.3
// proofs/s in flight (DESIGN.md §13 "Wider windows", profiles/r06/wide/)
int choose_c(uint64_t npts) {
  int lg = 0;
  while ((1ull << lg) < npts) lg++;
  int cc = lg - 4;
  if (cc < 7) cc = 7;  // staging LDS of the partition pass: 256 * 2 * ceil(255/c) * 7 B <= 133 KB
  if (cc > 17) cc = 17;
  if (const char* e = getenv("KGS_MSM_C")) {  // A/B override of the window
    int v = atoi(e);
    if (v >= 7 && v <= KGS_C_MAX) cc = v;
  }
  return cc;
}

// MSM work buffers of both lanes, for MSMs of up to npts points with window c
void ensure_msm_work(kgs_ctx& c) {
  const uint64_t npts = c.tb.npts;
  if (c.work_npts >= npts && c.work_npts) return;
  c.work_npts = 0;  // invalid until every buffer below exists
  const int cc = c.tb.c, W = c.tb.W;
  const uint64_t E = npts * W;
  const uint32_t B = 1u << (cc - 1);
  uint64_t nseg = (1ull << 18) + (1ull << 16) + 2;
  if (E / 64 + 2 > nseg) nseg = E / 64 + 2;
  c.msm_nseg_max = nseg;
  for (int lane = 0; lane < 2; lane++) {
    MsmWork& w = lane ? c.mw2 : c.mw;
    const std::string sfx = lane ? "_2" : "";
    w.digit = (int32_t*)c.buf("msm_digit" + sfx, E * 4);
    w.sorted = c.buf("msm_sorted" + sfx, E * 4);
    w.lo = (uint8_t*)c.buf("msm_lo" + sfx, E);
    const size_t NH = (size_t)msm_nh(cc);
    w.blockhist = c.buf("msm_blockhist" + sfx, 4 * (NH + 8) * ((npts + 255) / 256 + 1));
    w.counts = c.buf("msm_counts" + sfx, 4 * (NH + 300));
    w.offsets = c.buf("msm_offsets" + sfx, 4 * (B + 4));
    // hi_off (NH + 1), cpre (NH + 1) at MSM_NH_MAX + 8 words each, then the lo pass's block ->
    // partition table (at most NH + E / 16384 chunks: msm.hip chunk_bound)
    w.cursor = c.buf("msm_cursor" + sfx, 4 * (2 * ((size_t)MSM_NH_MAX + 8) + NH + E / 16384 + 64));
    w.segowner = c.buf("msm_segowner" + sfx, 4 * nseg);
    w.locnt = c.buf("msm_locnt" + sfx, 4 * NH * 256 * (size_t)MSM_SL_G_MAX);  // partitions x lo x chunks
    w.chunklist = c.buf("msm_chunklist" + sfx, 4 * 3 * (nseg / 16 + B + 16));
    w.chunkcnt = c.buf("msm_chunkcnt" + sfx, 64);
    w.raw29 = c.buf("msm_raw29" + sfx, 160 * ((size_t)B + 2 + nseg));
    w.part = c.buf("msm_part" + sfx, 160 * (size_t)(2 << (cc / 2)));  // row + column sums
  }
  c.work_npts = npts;
}

// Build (or share) the window tables of `npts` LEM points. `file` identifies the source; an empty
// `file` (in-memory points) is never shared. (srank, sworld): the points are a rank's slice of the
// SRS (points srank + sworld * j of the file; sworld == 1: the prefix). The context's SRS is replaced
// only once the new tables and the work buffers exist: a failed load leaves the context without an
// SRS ("no SRS loaded"), never with a half-built one. The device registry lock is held only to look
// up and to publish: the build (H2D copy + window expansion, seconds at 2^25 points) runs outside it,
// so other contexts of the device are not blocked meanwhile; a concurrent build of the same tables
// that published first wins and this one is dropped.
static std::shared_ptr<SrsTables> srs_lookup(int device, const std::string& file, int nbits_max, int srank, int sworld) {
  if (file.empty()) return nullptr;
  for (auto& w : g_srs_reg) {
    auto t = w.lock();
    if (t && t->device == device && t->file == file && t->nbits_max >= nbits_max && t->slice_rank == srank &&
        t->slice_world == sworld)
      return t;
  }
  return nullptr;
}

void load_points(kgs_ctx& c, const uint8_t* lem, uint64_t npts, int power, int nbits_max, const std::string& file,
                 int srank = 0, int sworld = 1) {
  if (npts < 2) throw KgsError(KGS_E_ARG, "SRS needs at least 2 points");
  c.sync();
  c.use_srs(nullptr);
  c.work_npts = 0;
  std::shared_ptr<SrsTables> s;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    s = srs_lookup(c.device, file, nbits_max, srank, sworld);
  }
  if (!s) {
    int cc = choose_c(npts);
    int W = (255 + cc - 1) / cc;
    // sorted entries pack j * npts + i into 31 bits (bit 31 = sign): widen the window until it fits
    while ((uint64_t)W * npts > (1ull << 31) && cc < KGS_C_MAX) {
      cc++;
      W = (255 + cc - 1) / cc;
    }
    if ((uint64_t)W * npts > (1ull << 31)) throw KgsError(KGS_E_SRS, "SRS too large for the MSM entry index");
    auto t = std::make_shared<SrsTables>();
    t->device = c.device;
    t->file = file;
    t->power = power;
    t->nbits_max = nbits_max;
    t->slice_rank = srank;
    t->slice_world = sworld;
    t->tb.npts = npts;
    t->tb.c = cc;
    t->tb.W = W;
    HC(dev_malloc((void**)&t->tb.table, (size_t)W * npts * 64));
    HC(hipMemcpyAsync(t->tb.table, lem, npts * 64, hipMemcpyHostToDevice, c.st));
    // build temporaries are released right after the build (they would otherwise stay in the pool)
    struct Tmp {
      void* p = nullptr;
      ~Tmp() {
        if (p) hipFree(p);
      }
    } tmp, scr;
    HC(dev_malloc(&tmp.p, npts * 128));
    HC(dev_malloc(&scr.p, npts * 32));
    msm_build_table(c.st, t->tb.table, npts, cc, W, (uint32_t*)tmp.p, (uint32_t*)scr.p);
    check_launch();
    HC(hipStreamSynchronize(c.st));
    std::lock_guard<std::mutex> lk(g_reg_mu);
    if (auto other = srs_lookup(c.device, file, nbits_max, srank, sworld)) {
      s = other;  // built concurrently by another context and published first: ours is released
    } else {
      g_srs_reg.erase(std::remove_if(g_srs_reg.begin(), g_srs_reg.end(), [](auto& w) { return w.expired(); }),
                      g_srs_reg.end());
      if (!file.empty()) g_srs_reg.push_back(t);
      s = t;
    }
  }
  ensure_domain(c, s->nbits_max + 1);
  MsmTables keep = c.tb;
  c.tb = s->tb;  // ensure_msm_work sizes from the new tables
  try {
    ensure_msm_work(c);
  } catch (...) {
    c.tb = keep;
    c.use_srs(nullptr);
    throw;
  }
  c.sync();
  c.use_srs(s);
}

// ------------------------------------------------------------------ MSM (commit)
// Polynomial.multiExponentiation (polynomial.js:1106-1115): device Pippenger -> c bit-sum points
// T_k (XYZZ) -> host sum_k 2^k T_k -> affine LEM. Sharded (world > 1): this rank's point range
// only; the partials of all ranks are all-gathered once per batch of commits (one prover round).

// The host-boundary copy streams (st_copy: input DMAs, st_wb: the Montgomery write-back) carry only
// copies and event waits. HIP maps streams onto a few hardware queues per priority level
// (GPU_MAX_HW_QUEUES, 4 by default), so with several contexts in flight a copy stream would share a
// hardware queue with another proof's compute stream, whose kernels then queue behind the copy
// stream's waits. Created at the lowest priority they get their own pool of hardware queues
// (KGS_COPY_STREAM_PRIO=normal keeps them in the compute streams' pool, for A/B).
hipStream_t copy_stream() {
  static const bool low = [] {
    const char* e = getenv("KGS_COPY_STREAM_PRIO");
    return !(e && !strcmp(e, "normal"));
  }();
  hipStream_t s = nullptr;
  if (low) {
    int least = 0, greatest = 0;
    HC(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HC(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least));
  } else {
    HC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  return s;
}

void shard_range(uint64_t n, int rank, int world, uint64_t& lo, uint64_t& hi) {
  lo = (uint64_t)((unsigned __int128)n * (unsigned)rank / (unsigned)world);
  hi = (uint64_t)((unsigned __int128)n * (unsigned)(rank + 1) / (unsigned)world);
}

// `to` waits for everything issued so far on `from` (lane hand-over inside a round)
void lane_join(kgs_ctx& c, hipStream_t from, hipStream_t to) {
  if (from == to) return;
  if (!c.ev_join) HC(hipEventCreateWithFlags(&c.ev_join, hipEventDisableTiming));
  HC(hipEventRecord(c.ev_join, from));
  HC(hipStreamWaitEvent(to, c.ev_join, 0));
}

// the second MSM lane starts after everything issued so far on the main stream (the round's inputs)
void fork_lanes(kgs_ctx& c) {
  if (c.msm_lanes < 2) return;
  if (!c.st2) {
    HC(hipStreamCreateWithFlags(&c.st2, hipStreamNonBlocking));
    HC(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
  }
  HC(hipEventRecord(c.ev_fork, c.st));
  HC(hipStreamWaitEvent(c.st2, c.ev_fork, 0));
}

Commit commit_launch_slice(kgs_ctx& c, const uint32_t* scalars, uint64_t count, uint64_t pbase, uint64_t pstride,
                           uint64_t N, int slot, int lane) {
  Commit cm;
  cm.N = N;
  const int cc = c.tb.c;
  const int slots = c.msm_slots > 64 ? c.msm_slots : 64;
  if (slot >= slots) throw KgsError(KGS_E_ARG, "too many commitments in flight");
  uint64_t cap = c.tb.npts;  // global points the resident SRS covers
  if (c.srs_slice_world > 1) {
    // a rank's SRS slice holds the points slice_rank + slice_world * j only: it serves exactly the
    // commitments over this rank's CYCLIC slice, whose scalar j multiplies that point
    if (count && (pstride != (uint64_t)c.srs_slice_world || pbase != (uint64_t)c.srs_slice_rank))
      throw KgsError(KGS_E_ARG, "the loaded SRS slice (rank " + std::to_string(c.srs_slice_rank) + " of " +
                                    std::to_string(c.srs_slice_world) + ") does not hold this commitment's points");
    pbase = 0;
    pstride = 1;
    cap = (uint64_t)c.srs_slice_rank + (uint64_t)c.srs_slice_world * c.tb.npts;
  }
  if (N > cap || (count && pbase + pstride * (count - 1) >= c.tb.npts))
    throw KgsError(KGS_E_SRS, "MSM larger than the resident SRS");
  uint32_t* dT = c.buf("msm_T", (size_t)slots * cc * 128) + (size_t)slot * cc * 32;
  cm.h_T = c.pin((size_t)cc * 128);
  if (count == 0) {
    memset(cm.h_T, 0, (size_t)cc * 128);  // ZZ == 0: infinity
    return cm;
  }
  if (c.msm_lanes < 2) lane = 0;
  hipStream_t st = lane ? c.st2 : c.st;  // lane 1 was forked (fork_lanes) after the round's inputs
  msm_run(st, c.tb, lane ? c.mw2 : c.mw, scalars, count, dT, nullptr, pbase, pstride, c.msm_lanes >= 2);
  check_launch();
  HC(hipMemcpyAsync(cm.h_T, dT, (size_t)cc * 128, hipMemcpyDeviceToHost, st));
  return cm;
}

// MSM point-range sharding (kgs_ctx_set_shard): this rank's contiguous range of the N points
Commit commit_launch(kgs_ctx& c, const uint32_t* scalars, uint64_t N, int slot, int lane) {
  uint64_t lo = 0, hi = N;
  if (c.shard_world > 1) shard_range(N, c.shard_rank, c.shard_world, lo, hi);
  Commit cm = commit_launch_slice(c, scalars + (size_t)8 * lo, hi - lo, lo, 1, N, slot, lane);
  return cm;
}

bool split_commits(const kgs_ctx& c) { return c.msm_lanes >= 2 && c.shard_world == 1; }

Commit commit_launch_split(kgs_ctx& c, const uint32_t* scalars, uint64_t N, uint64_t cut, int slot) {
  if (!split_commits(c) || cut == 0 || cut >= N) return commit_launch(c, scalars, N, slot, 0);
  Commit a = commit_launch_slice(c, scalars, cut, 0, 1, N, slot, 0);
  Commit b = commit_launch_slice(c, scalars + (size_t)8 * cut, N - cut, cut, 1, N, slot + 1, 1);
  a.h_T2 = b.h_T;
  return a;
}

// sum_k 2^k sum_r T_k^(r) -> affine LEM
void combine_partials(const uint8_t* T_all, size_t part_stride, int nparts, int cc, uint8_t out[64]) {
  host::G1 acc = host::G1::inf();
  for (int k = cc - 1; k >= 0; k--) {
    acc = acc.dbl();
    for (int r = 0; r < nparts; r++) acc = acc.add(host::G1::from_bytes128(T_all + r * part_stride + 128 * k));
  }
  acc.to_affine_lem(out);
}

// after sync: finish a batch of commits; with world > 1 the partials of all ranks are exchanged in
// ONE all-gather per batch (one prover round) and summed on the host
void commits_finish_with(kgs_ctx& c, const std::vector<Commit>& cms, std::vector<uint8_t*> outs, int world,
                         const HostAllgather& ag) {
  const int cc = c.tb.c;
  const size_t tb = (size_t)cc * 128;
  bool any = false;
  for (auto& cm : cms) any |= cm.N > 0;
  if (world == 1 || !any) {
    std::vector<uint8_t> two;
    for (size_t i = 0; i < cms.size(); i++) {
      if (cms[i].N && cms[i].h_T2) {  // split over the two lanes: both partials
        two.resize(2 * tb);
        memcpy(two.data(), cms[i].h_T, tb);
        memcpy(two.data() + tb, cms[i].h_T2, tb);
        combine_partials(two.data(), tb, 2, cc, outs[i]);
      } else if (cms[i].N) {
        combine_partials(cms[i].h_T, tb, 1, cc, outs[i]);
      } else {
        host::G1::inf().to_affine_lem(outs[i]);
      }
    }
    return;
  }
  const size_t bytes = tb * cms.size();
  std::vector<uint8_t> send(bytes), recv(bytes * world);
  for (size_t i = 0; i < cms.size(); i++) memcpy(send.data() + i * tb, cms[i].h_T, tb);
  ag(send.data(), recv.data(), bytes);
  for (size_t i = 0; i < cms.size(); i++) {
    if (cms[i].N) combine_partials(recv.data() + i * tb, bytes, world, cc, outs[i]);
    else host::G1::inf().to_affine_lem(outs[i]);
  }
}

void commits_finish(kgs_ctx& c, const std::vector<Commit>& cms, std::vector<uint8_t*> outs) {
  commits_finish_with(c, cms, outs, c.shard_world, [&](const void* send, void* recv, size_t bytes) {
    if (!c.shard_fn) throw KgsError(KGS_E_COMM, "sharding enabled without an all-gather callback");
    if (c.shard_fn(c.shard_user, (const uint8_t*)send, (uint8_t*)recv, bytes) != 0)
      throw KgsError(KGS_E_COMM, "shard all-gather failed");
  });
}

void commit_finish(kgs_ctx& c, const Commit& cm, uint8_t out[64]) { commits_finish(c, {cm}, {out}); }

// ------------------------------------------------------------------ Horner evaluation
// returns p_j(x) for each poly of the batch

// The 29-bit product record of a constant (fr29.hpp mul29): x * 2^261 mod r (x's Montgomery form times
// 32) in 9 x 29-bit limbs + zero pad, as two 32-byte scalar slots; the per-element kernels multiply by
// a uniform constant with it (one mad per partial product, no carry words)
void fr29_record(const Fr& x, Fr out[2]) {
  const Fr y = x * Fr::from_u64(32);
  uint32_t w[16] = {0};
  for (int j = 0; j < 9; j++) {
    const int bit = 29 * j, i = bit >> 6, off = bit & 63;
    uint64_t l = y.v[i] >> off;
    if (off > 35 && i + 1 < 4) l |= y.v[i + 1] << (64 - off);
    w[j] = (uint32_t)(l & 0x1fffffffu);
  }
  memcpy(out[0].v, w, 32);
  memcpy(out[1].v, w + 8, 32);
}

// xp[l] = x^(8 * 2^l) (l < 8), xp[8] = x, xp[9] = x^2048, xp[10..11] = the 29-bit record of x,
// xp[12 + 2l .. 13 + 2l] = the record of xp[l] (l < 8)
uint32_t* xpowers(kgs_ctx& c, const Fr& x) {
  Fr p[28];
  Fr x8 = x.sqr().sqr().sqr();
  p[0] = x8;
  for (int l = 1; l < 8; l++) p[l] = p[l - 1].sqr();
  p[8] = x;
  p[9] = p[7].sqr();  // x^2048
  fr29_record(x, p + 10);
  for (int l = 0; l < 8; l++) fr29_record(p[l], p + 12 + 2 * l);
  return c.scal(p, 28);
}

EvalJob eval_launch(kgs_ctx& c, const std::vector<const uint32_t*>& src, const std::vector<uint64_t>& len, const Fr& x,
                    int slot) {
  EvalJob j;
  j.src = src;
  j.len = len;
  j.x = x;
  uint64_t maxlen = 1;
  for (auto l : len) maxlen = l > maxlen ? l : maxlen;
  j.ntiles = (uint32_t)((maxlen + EVAL_TILE - 1) / EVAL_TILE);
  const int np = (int)src.size();
  uint32_t* xp = xpowers(c, x);
  size_t bytes = (size_t)32 * j.ntiles * (np ? np : 1);
  uint32_t* dpart = c.buf("eval_part_" + std::to_string(slot), bytes);
  // batches of EB_MAX polynomials per launch (any number of multisets), partials contiguous per poly
  for (int p0 = 0; p0 < np; p0 += EB_MAX) {
    EvalBatch eb;
    eb.npolys = np - p0 < EB_MAX ? np - p0 : EB_MAX;
    for (int i = 0; i < eb.npolys; i++) {
      eb.src[i] = src[p0 + i];
      eb.len[i] = len[p0 + i];
    }
    launch_eval_tiles(c.st, dpart + (size_t)8 * j.ntiles * p0, eb, xp, j.ntiles);
    check_launch();
  }
  j.h_part = c.pin(bytes);
  HC(hipMemcpyAsync(j.h_part, dpart, bytes, hipMemcpyDeviceToHost, c.st));
  return j;
}

std::vector<Fr> eval_finish(const EvalJob& j) {
  Fr X = j.x;
  for (int i = 0; i < 11; i++) X = X.sqr();  // x^2048
  std::vector<Fr> out;
  for (size_t p = 0; p < j.src.size(); p++) {
    Fr v = Fr::zero();
    for (uint32_t b = j.ntiles; b-- > 0;) v = v * X + Fr::from_bytes(j.h_part + 32 * ((size_t)p * j.ntiles + b));
    out.push_back(v);
  }
  return out;
}

// ------------------------------------------------------------------ the prover


void run_lincomb(hipStream_t st, uint32_t* out, uint64_t n, const LcTerms& t) {
  size_t k = 0;
  bool first = true;
  do {
    LinComb lc{};
    if (!first) {
      lc.src[0] = out;
      lc.len[0] = n;
      Fr::one().to_bytes((uint8_t*)lc.coef[0]);
      Fr rec[2];
      fr29_record(Fr::one(), rec);
      memcpy(lc.coef29[0], rec, 4 * LC_W29);
      lc.nterms = 1;
    }
    for (; k < t.src.size() && lc.nterms < LC_MAX; k++) {
      lc.src[lc.nterms] = t.src[k];
      lc.len[lc.nterms] = t.len[k];
      t.coef[k].to_bytes((uint8_t*)lc.coef[lc.nterms]);
      Fr rec[2];
      fr29_record(t.coef[k], rec);
      memcpy(lc.coef29[lc.nterms], rec, 4 * LC_W29);
      lc.nterms++;
    }
    (first ? t.c0 : Fr::zero()).to_bytes((uint8_t*)lc.c0);
    launch_lincomb(st, out, n, lc);
    check_launch();
    first = false;
  } while (k < t.src.size());
}

// Round 5 (prover.js:320-413): r(X) + the opening numerator as sum_k coef_k P_k + c0, from the
// challenges and round-4 evaluations. Z_H(xi), L1(xi) as polynomial_utils.js:1-19. Shared by the
// single-GPU and the distributed prover.
R5 round5_terms(bool gs, bool sel, int k, int nbits, const Fr& alpha, const Fr& beta, const Fr& gamma, const Fr& v,
                const Fr& xi, const std::vector<Fr>& fx, const std::vector<Fr>& tx, const Fr& sFx, const Fr& sTx,
                const Fr& sxiw, bool lookup, const Fr* fxi_override) {
  const uint64_t n = 1ull << nbits;
  Fr xn = xi;
  for (int i = 0; i < nbits; i++) xn = xn.sqr();
  const Fr zh = xn - Fr::one();
  const Fr l1 = zh * (Fr::from_u64(n) * (xi - Fr::one())).inverse();
  Fr fxi = Fr::zero(), txi = Fr::zero();
  for (int i = k - 1; i >= 0; i--) {
    fxi = fxi * beta + fx[i];
    if (gs) txi = txi * beta + tx[i];
  }
  if (fxi_override) fxi = *fxi_override;
  const Fr one = Fr::one();
  Fr selBin = Fr::zero();  // alpha^3 selTBin + alpha^2 selFBin (a lookup has no selTBin term)
  if (sel) selBin = ((lookup ? Fr::zero() : (sTx - sTx.sqr()) * alpha) + (sFx - sFx.sqr())) * alpha * alpha;
  std::vector<Fr> vp(2 * k + 4);
  vp[0] = one;
  for (size_t i = 1; i < vp.size(); i++) vp[i] = vp[i - 1] * v;
  R5 r;
  Fr c0;
  if (gs) {
    const Fr fg = fxi + gamma, tg = txi + gamma;
    Fr rc = sxiw * fg * tg + (sel ? sTx * fg - sFx * tg : fxi - txi);
    c0 = selBin + alpha * rc;
    r.terms.push_back({R5_S, 0, l1 - alpha * fg * tg});
    r.terms.push_back({R5_Q, 0, zh.neg()});
    for (int i = 0; i < k; i++) {
      r.terms.push_back({R5_F, i, vp[1 + i]});
      c0 = c0 - vp[1 + i] * fx[i];
    }
    for (int i = 0; i < k; i++) {
      r.terms.push_back({R5_T, i, vp[1 + k + i]});
      c0 = c0 - vp[1 + k + i] * tx[i];
    }
    if (sel) {
      r.terms.push_back({R5_SELF, 0, vp[2 * k + 1]});
      r.terms.push_back({R5_SELT, 0, vp[2 * k + 2]});
      c0 = c0 - vp[2 * k + 1] * sFx - vp[2 * k + 2] * sTx;
    }
  } else {
    const Fr fg = fxi + gamma;
    const Fr dF = sel ? sFx * (fg - one) + one : fg;
    c0 = selBin + alpha * sxiw * (sel ? sTx * (gamma - one) + one : gamma) - l1;
    r.terms.push_back({R5_POLT, 0, alpha * sxiw * (sel ? sTx : one)});
    r.terms.push_back({R5_S, 0, l1 - alpha * dF});
    r.terms.push_back({R5_Q, 0, zh.neg()});
    for (int i = 0; i < k; i++) {
      r.terms.push_back({R5_F, i, vp[1 + i]});
      c0 = c0 - vp[1 + i] * fx[i];
    }
    if (sel) {
      r.terms.push_back({R5_SELF, 0, vp[k + 1]});
      r.terms.push_back({R5_SELT, 0, vp[k + 2]});
      c0 = c0 - vp[k + 1] * sFx - vp[k + 2] * sTx;
    }
  }
  r.c0 = c0;
  return r;
}

void prove_impl(kgs_ctx& c, const ProveIn& in, uint8_t* com_out, uint8_t* ev_out) {
  if (in.kind != KGS_GRANDSUM && in.kind != KGS_GRANDPRODUCT && in.kind != KGS_LOOKUP)
    throw KgsError(KGS_E_ARG, "unknown argument kind");
  if (in.kind == KGS_LOOKUP && !in.sel_f)
    throw KgsError(KGS_E_ARG, "a lookup needs both selectors (sel_t holds the multiplicities)");
  c.xs.reset();
  ensure_twin(c);  // a domain last grown by a quirks replay has no 29-bit twin yet
  if (c.group) {
    prove_dist_group(c, in, com_out, ev_out);
    return;
  }
  // in-flight contexts (one MSM lane) launch the NTT passes built to co-reside with the other proofs'
  // accumulate waves, the latency mode (two lanes) the build that is fastest alone (ntt.hip, WV)
  struct NttMode {
    bool prev;
    explicit NttMode(bool on) : prev(ntt_set_coresident(on)) {}
    ~NttMode() { ntt_set_coresident(prev); }
  } ntt_mode(c.msm_lanes < 2);
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  // every slot, the host-boundary ones [6..8] too: kgs_prove writes them after this returns, and a
  // device-resident proof must not report a previous host call's copy and prover times
  c.timing.assign(9, 0.0);
  Range range(ROUND_NAMES[0]);
  auto lap = [&](int r) {
    auto t1 = clk::now();
    c.timing[r] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    t0 = t1;
    if (r + 1 < 5) range.push(ROUND_NAMES[r + 1]);
    else range.pop();
  };
  const bool gs = in.kind != KGS_GRANDPRODUCT;  // KGS_LOOKUP is a selected grand-sum
  const bool lk = in.kind == KGS_LOOKUP;
  const bool sel = in.sel_f != nullptr;
  const int k = in.npols;
  const int nbits = in.nbits;
  const uint64_t n = 1ull << nbits;
  const size_t E = 32 * n;
  if (nbits < 1) throw KgsError(KGS_E_ARG, "nbits must be >= 1");
  if (c.srs_power < 0) throw KgsError(KGS_E_ARG, "no SRS loaded");
  if (c.srs_slice_world > 1)
    throw KgsError(KGS_E_ARG, "this context holds a rank's SRS slice: it proves only as that rank of a group (kgs_ctx_set_group)");
  if (c.srs_power < nbits)
    throw KgsError(KGS_E_SRS, "The Powers of Tau file is not sufficiently large to commit the polynomials.");
  if (nbits > c.nbits_max) throw KgsError(KGS_E_SRS, "SRS loaded for a smaller maximum domain; reload with larger nbits_max");
  if (k < 1) throw KgsError(KGS_E_ARG, "The number of multisets must be greater than 0.");
  if (k > KGS_MAX_POLS) throw KgsError(KGS_E_ARG, "too many multisets");
  // pinned staging for this proof's host round trips: commit partials (c x 128 B each), the
  // round-4 Horner tile partials (32 B per 2048 coefficients per evaluated polynomial), flags and
  // scalars (each bump allocation rounds up to 64 B)
  const int ncom_all = 2 * k + (in.sel_f ? 2 : 0) + 4;
  c.msm_slots = ncom_all + 4;
  {
    const size_t ntl = (size_t)((n + EVAL_TILE - 1) / EVAL_TILE);
    const size_t need = (size_t)(ncom_all + 4) * ((size_t)c.tb.c * 128 + 64) + 32 * ntl * (2 * k + 3) + 64 * 8 +
                        ((size_t)kgs_ctx::SCAL_BYTES * 2) + (1 << 20);
    c.ensure_pin(need > ((size_t)8 << 20) ? need : ((size_t)8 << 20));
  }
  c.reset_staging();
  uint32_t* flags = c.buf("flags", 64);
  HC(hipMemsetAsync(flags, 0, 64, c.st));
  const bool vec = k > 1;

  // ---------------- round 1: witness polynomials + commitments (prover.js:144-179)
  std::vector<uint32_t*> fm(k), tm(k), Fc(k), Tc(k);
  for (int i = 0; i < k; i++) {
    fm[i] = c.buf("fm" + std::to_string(i), E);
    tm[i] = c.buf("tm" + std::to_string(i), E);
    Fc[i] = c.buf("Fc" + std::to_string(i), E);
    Tc[i] = c.buf("Tc" + std::to_string(i), E);
  }
  uint32_t *sFc = nullptr, *sTc = nullptr;
  if (sel) {
    sFc = c.buf("sFc", E);
    sTc = c.buf("sTc", E);
  }
  // Host-buffer inputs (kgs_prove) arrive vector by vector: in.input_issued(v) returns once vector
  // v's DMA is enqueued (its host copy may still be running on another thread before that), and
  // in.ready[v] is the event its first kernel waits for.
  auto wait_input = [&](size_t v, hipStream_t st) {
    if (in.input_issued) in.input_issued(v);
    if (v < in.ready.size() && in.ready[v]) HC(hipStreamWaitEvent(st, in.ready[v], 0));
  };
  // Montgomery write-back (prover.js:147-148): vector v's D2H on the write-back stream right after
  // its conversion on `st` (not after the round's MSMs, and never queued between input DMAs)
  int nwb = 0;
  auto write_back = [&](uint8_t* dst, const uint32_t* src, hipStream_t st) {
    if (!dst) return;
    if (!c.st_wb) c.st_wb = copy_stream();
    if ((int)c.ev_wb.size() <= nwb) {
      hipEvent_t e;
      HC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      c.ev_wb.push_back(e);
    }
    HC(hipEventRecord(c.ev_wb[nwb], st));
    HC(hipStreamWaitEvent(c.st_wb, c.ev_wb[nwb], 0));
    nwb++;
    // hipMemcpyAsync. Into pinned memory the runtime runs it as its copyBuffer shader kernel, not on an
    // SDMA engine: ~0.8 ms of CU residency per 32 MiB in flight; hipMemcpyDtoHAsync does the same
    // (profiles/r06/host_engine/, wb_api/). KGS_WB_COPY=kernel stores from our own shader into the
    // mapped pinned buffer instead (poly.hip k_host_store): measured slower in flight, 83-85 vs 86-88
    // proofs/s (profiles/r05/wb_ab.txt), kept for A/B
    static const unsigned wb_blocks = [] {
      const char* e = getenv("KGS_WB_COPY");
      if (!(e && !strcmp(e, "kernel"))) return 0u;
      const char* b = getenv("KGS_WB_BLOCKS");
      return b ? (unsigned)atoi(b) : 64u;
    }();
    void* mapped = nullptr;
    if (wb_blocks && hipHostGetDevicePointer(&mapped, dst, 0) != hipSuccess) {
      (void)hipGetLastError();
      mapped = nullptr;
    }
    if (mapped && E % 16 == 0) launch_host_store(c.st_wb, mapped, src, E, wb_blocks);
    else HC(hipMemcpyAsync(dst, src, E, hipMemcpyDeviceToHost, c.st_wb));
  };
  auto mont_out = [&](const std::vector<uint8_t*>& v, int i) -> uint8_t* { return v.empty() ? nullptr : v[i]; };
  std::vector<Commit> r1;
  int slot = 0;
  // With two MSM lanes (a proof alone on its context: the latency mode) each input vector's whole
  // round-1 chain — Montgomery conversion, iNTT, commitment MSM — runs on the lane of its
  // commitment, F_i / selF on lane 0 and T_i / selT on lane 1, so that T's transfer (host buffers)
  // and T's transform overlap F's MSM instead of delaying it.
  const bool piped = split_commits(c);
  if (piped) {
    fork_lanes(c);
    for (int i = 0; i < k; i++) {
      wait_input(2 * i, c.st);
      launch_to_mont(c.st, fm[i], in.f_std[i], n);
      write_back(mont_out(in.mont_f_out, i), fm[i], c.st);
      intt_nat(c, Fc[i], fm[i], nbits);
      r1.push_back(commit_launch(c, Fc[i], n, slot++, 0));
      wait_input(2 * i + 1, c.st2);
      launch_to_mont(c.st2, tm[i], in.t_std[i], n);
      write_back(mont_out(in.mont_t_out, i), tm[i], c.st2);
      intt_nat(c, Tc[i], tm[i], nbits, c.st2);
      r1.push_back(commit_launch(c, Tc[i], n, slot++, 1));
    }
    check_launch();
  } else {
    for (int i = 0; i < k; i++) {
      wait_input(2 * i, c.st);
      launch_to_mont(c.st, fm[i], in.f_std[i], n);
      write_back(mont_out(in.mont_f_out, i), fm[i], c.st);
      wait_input(2 * i + 1, c.st);
      launch_to_mont(c.st, tm[i], in.t_std[i], n);
      write_back(mont_out(in.mont_t_out, i), tm[i], c.st);
      intt_nat(c, Fc[i], fm[i], nbits);
      intt_nat(c, Tc[i], tm[i], nbits);
    }
    check_launch();
  }
  // fm/tm are not written again before the round-1 sync (the write-back reads them on st_wb)
  if (sel) {
    if (piped) {
      wait_input(2 * k, c.st);
      intt_nat(c, sFc, in.sel_f, nbits);
      r1.push_back(commit_launch(c, sFc, n, slot++, 0));
      wait_input(2 * k + 1, c.st2);
      intt_nat(c, sTc, in.sel_t, nbits, c.st2);
      r1.push_back(commit_launch(c, sTc, n, slot++, 1));
    } else {
      wait_input(2 * k, c.st);
      intt_nat(c, sFc, in.sel_f, nbits);
      wait_input(2 * k + 1, c.st);
      intt_nat(c, sTc, in.sel_t, nbits);
    }
  }
  if (!piped) {
    fork_lanes(c);
    for (int i = 0; i < k; i++) {
      r1.push_back(commit_launch(c, Fc[i], n, slot++, 0));
      r1.push_back(commit_launch(c, Tc[i], n, slot++, 1));
    }
    if (sel) {
      r1.push_back(commit_launch(c, sFc, n, slot++, 0));
      r1.push_back(commit_launch(c, sTc, n, slot++, 1));
    }
  }
  // round 1's commitments only: the Montgomery write-back on st_wb keeps running under rounds 2-5
  // (in.after_round1's thread waits for it before copying to the caller)
  HC(hipStreamSynchronize(c.st));
  if (c.st2) HC(hipStreamSynchronize(c.st2));
  if (in.after_round1) in.after_round1();
  const int ncom = 2 * k + (sel ? 2 : 0) + 4;
  std::vector<std::vector<uint8_t>> com(ncom, std::vector<uint8_t>(64));
  int ci = 0;
  {
    std::vector<uint8_t*> outs;
    for (size_t i = 0; i < r1.size(); i++) outs.push_back(com[ci++].data());
    commits_finish(c, r1, outs);
  }
  lap(0);

  // ---------------- round 2: challenges, combined polynomials, S / Z (prover.js:181-231)
  host::Transcript tr;
  for (int i = 0; i < ci; i++) tr.add_commitment(com[i].data());
  Fr beta = Fr::zero();
  if (vec) {
    beta = tr.challenge();
    tr.add_scalar(beta);
  }
  const Fr gamma = tr.challenge();
  std::vector<Fr> bpow(k);
  bpow[0] = Fr::one();
  for (int i = 1; i < k; i++) bpow[i] = bpow[i - 1] * beta;
  // Two lanes (latency mode): the challenge-independent coset evaluations of F, T (+ selectors) run on
  // lane 1 from the start of the round, beside the builder's serial part (k_tile_inverse is one
  // workgroup) and S's inverse NTT on lane 0; S's commitment follows on lane 0, S's coset evaluation
  // on lane 1 once S exists. One lane: the same work in order on the main stream.
  fork_lanes(c);
  hipStream_t s2 = c.msm_lanes >= 2 && c.st2 ? c.st2 : c.st;
  const int lcs = (!gs && !sel) ? nbits : nbits + 1;
  const uint64_t cs = 1ull << lcs;
  uint32_t* cosS = c.buf("cosS", 32 * cs);
  uint32_t* cosF = c.buf("cosF", 32 * cs);
  uint32_t* cosT = c.buf("cosT", 32 * cs);
  uint32_t *cosSF = nullptr, *cosST = nullptr;
  const uint32_t *fcomb = fm[0], *tcomb = tm[0], *polF = Fc[0], *polT = Tc[0];
  if (vec) {
    uint32_t* b_fe = c.buf("fcomb", E);
    uint32_t* b_te = c.buf("tcomb", E);
    uint32_t* b_F = c.buf("polF", E);
    uint32_t* b_T = c.buf("polT", E);
    LcTerms l1, l2, l3, l4;
    for (int i = 0; i < k; i++) {
      l1.add(fm[i], n, bpow[i]);
      l2.add(tm[i], n, bpow[i]);
      l3.add(Fc[i], n, bpow[i]);
      l4.add(Tc[i], n, bpow[i]);
    }
    run_lincomb(c.st, b_fe, n, l1);
    run_lincomb(c.st, b_te, n, l2);
    run_lincomb(s2, b_F, n, l3);
    run_lincomb(s2, b_T, n, l4);
    fcomb = b_fe;
    tcomb = b_te;
    polF = b_F;
    polT = b_T;
  }
  coset_fwd(c, cosF, polF, n, lcs, s2);
  coset_fwd(c, cosT, polT, n, lcs, s2);
  if (sel) {
    cosSF = c.buf("cosSF", 32 * cs);
    cosST = c.buf("cosST", 32 * cs);
    coset_fwd(c, cosSF, sFc, n, lcs, s2);
    coset_fwd(c, cosST, sTc, n, lcs, s2);
  }
  uint32_t* Sev = c.buf("Sev", E);
  uint32_t* Sc = c.buf("Sc", E);
  const uint32_t ntiles = (uint32_t)((n + EVAL_TILE - 1) / EVAL_TILE);
  uint32_t* d_gamma = c.scal(&gamma, 1);
  launch_builder(c.st, !gs, sel, Sev, fcomb, tcomb, in.sel_f, in.sel_t, d_gamma, n, c.buf("bt_tp", 32 * (ntiles + 1)),
                 c.buf("bt_ti", 32 * (ntiles + 1)), flags);
  intt_nat(c, Sc, Sev, nbits);
  check_launch();
  lane_join(c, c.st, s2);
  coset_fwd(c, cosS, Sc, n, lcs, s2);
  Commit cS = commit_launch(c, Sc, n, slot++, 0);
  uint32_t* nxm1 = get_nxm1(c, nbits, lcs);
  check_launch();
  uint32_t* h_flags = (uint32_t*)c.pin(64);
  HC(hipMemcpyAsync(h_flags, flags, 64, hipMemcpyDeviceToHost, c.st));
  c.sync();
  if (h_flags[0])
    throw KgsError(KGS_E_NOT_WELL_CALC, gs ? "The grand-sum polynomial S is not well calculated"
                                             : "The grand-product polynomial Z is not well calculated");
  const int iS = ci;
  commit_finish(c, cS, com[ci++].data());
  lap(1);

  // ---------------- round 3: quotient on a coset (prover.js:233-286)
  tr.add_scalar(gamma);
  tr.add_commitment(com[iS].data());
  const Fr alpha = tr.challenge();
  const uint32_t rot = (uint32_t)(cs >> nbits);
  uint64_t qlen = (!gs && !sel) ? n - 1 : 2 * n - 2;  // deg Q + 1 bound
  Fr gn = Fr::from_u64(5).pow_u64(n);
  // alpha_t: weight of the selT-binary term (none for a lookup, whose selT holds multiplicities)
  // 1/Z_H on the two coset halves, times 1/cs (the scaling of the inverse transform below; nxm1 carries it too)
  const Fr inv_cs = Fr::from_u64(cs).inverse();
  Fr qs[9] = {alpha, gamma, (gn - Fr::one()).inverse() * inv_cs, (gn.neg() - Fr::one()).inverse() * inv_cs,
              lk ? Fr::zero() : alpha};
  // k_quotient: alpha / Z_H on each coset half as one 29-bit product record (slots 5-6, 7-8)
  fr29_record(alpha * qs[2], qs + 5);
  fr29_record(alpha * qs[3], qs + 7);
  uint32_t* d_qs = c.scal(qs, 9);
  launch_divcheck(c.st, !gs, sel, flags + 1, Sev, fcomb, tcomb, in.sel_f, in.sel_t, d_qs, n);
  const uint32_t* Qc = c.buf("Qc", 32 * cs);
  launch_quotient(c.st, !gs, sel, (uint32_t*)Qc, cosS, cosF, cosT, cosSF, cosST, nxm1, d_qs, lcs, rot);
  coset_inv_prescaled(c, (uint32_t*)Qc, Qc, lcs);
  check_launch();
  // latency mode: Q's 2n points over both MSM lanes (one lane's sort and tail overlap the other's
  // accumulation)
  fork_lanes(c);
  Commit cQ = commit_launch_split(c, Qc, qlen, qlen / 2, slot);
  slot += 2;
  std::vector<const uint32_t*> qops = {polF, polT, Sc};
  if (sel) {
    qops.push_back(sFc);
    qops.push_back(sTc);
  }
  const uint32_t* probe = c.ref_quirks && !lk ? ref_quirks_probe(c, n, qops, Qc, qlen) : nullptr;
  HC(hipMemcpyAsync(h_flags, flags, 64, hipMemcpyDeviceToHost, c.st));
  c.sync();
  // Reference-quirks mode (ref_quirks.cpp): where the reference's own quotient chain does not compute
  // the quotient (an operand of degree 1 <= d < n/2) it is replayed with the reference's buffer
  // semantics and its Q replaces ours; otherwise the only difference is the reference's RangeError
  // on a zero quotient (divZh, after its divisibility check).
  const uint32_t* Fmut = nullptr;  // polF's buffer after the replay wrote into it (Q2), else nullptr
  bool replayed = false;
  if (probe) {
    if (ref_quirks_needed(probe, qops.size(), n)) {
      uint32_t* fm_out = nullptr;
      Qc = ref_quirks_quotient(c, gs, sel, lk, nbits, alpha, gamma, polF, polT, Sc, sFc, sTc, qlen, fm_out);
      Fmut = fm_out;
      replayed = true;
      // multiExponentiation reads degree()+1 points of the reference's 2n-point PTau buffer
      // (prover.js:83-84, polynomial.js:1106-1110); past it, ffjavascript's multiExpAffine gets fewer
      // bases than scalars, which is not reproduced
      if (qlen > 2 * n)
        throw KgsError(KGS_E_ARG, "reference-quirks mode: the reference's Q has more coefficients than its 2n-point SRS buffer");
      cQ = commit_launch_split(c, Qc, qlen, qlen / 2, slot);
      slot += 2;
      c.sync();
    }
  }
  if (!replayed) {
    if (h_flags[1]) throw KgsError(KGS_E_NOT_DIVISIBLE, "Polynomial is not divisible");
    if (probe && ref_quotient_is_zero(probe)) throw KgsError(KGS_E_RANGE, "offset is out of bounds");
  }
  const int iQ = ci;
  commit_finish(c, cQ, com[ci++].data());
  lap(2);

  // ---------------- round 4: evaluations (prover.js:288-318)
  tr.add_scalar(alpha);
  tr.add_commitment(com[iQ].data());
  const Fr xi = tr.challenge();
  const Fr w = fr_w(nbits);
  const Fr xiw = xi * w;
  std::vector<const uint32_t*> esrc;
  std::vector<uint64_t> elen;
  // reference-quirks mode, polF's buffer shared and rewritten (Q2): the reference's later reads of polF
  // see the new values — polFs[0] itself for one multiset, only polF.evaluate (prover.js:360) for vectors
  if (Fmut && !vec) Fc[0] = (uint32_t*)Fmut;
  for (int i = 0; i < k; i++) {
    esrc.push_back(Fc[i]);
    elen.push_back(n);
    if (gs) {
      esrc.push_back(Tc[i]);
      elen.push_back(n);
    }
  }
  if (sel) {
    esrc.push_back(sFc);
    elen.push_back(n);
    esrc.push_back(sTc);
    elen.push_back(n);
  }
  if (Fmut && vec) {
    esrc.push_back(Fmut);
    elen.push_back(n);
  }
  EvalJob ej1 = eval_launch(c, esrc, elen, xi, 0);
  EvalJob ej2 = eval_launch(c, {Sc}, {n}, xiw, 1);
  c.sync();
  std::vector<Fr> ev1 = eval_finish(ej1);
  const Fr sxiw = eval_finish(ej2)[0];
  std::vector<Fr> fx(k), tx(k);
  size_t p = 0;
  for (int i = 0; i < k; i++) {
    fx[i] = ev1[p++];
    if (gs) tx[i] = ev1[p++];
  }
  Fr sFx = Fr::zero(), sTx = Fr::zero();
  if (sel) {
    sFx = ev1[p++];
    sTx = ev1[p++];
  }
  const bool fxi_set = Fmut && vec;
  const Fr fxi_mut = fxi_set ? ev1[p++] : Fr::zero();
  std::vector<Fr> evals;  // proof order
  for (int i = 0; i < k; i++) {
    evals.push_back(fx[i]);
    if (gs) evals.push_back(tx[i]);
  }
  if (sel) {
    evals.push_back(sFx);
    evals.push_back(sTx);
  }
  evals.push_back(sxiw);
  lap(3);

  // ---------------- round 5: linearisation + openings (prover.js:320-413)
  tr.add_scalar(xi);
  for (int i = 0; i < k; i++) {
    tr.add_scalar(fx[i]);
    if (gs) tr.add_scalar(tx[i]);
  }
  if (sel) {
    tr.add_scalar(sFx);
    tr.add_scalar(sTx);
  }
  tr.add_scalar(sxiw);
  const Fr v = tr.challenge();
  const R5 r5 = round5_terms(gs, sel, k, nbits, alpha, beta, gamma, v, xi, fx, tx, sFx, sTx, sxiw, lk,
                             fxi_set ? &fxi_mut : nullptr);
  LcTerms lw;
  for (const R5Term& t : r5.terms) {
    switch (t.id) {
      case R5_S: lw.add(Sc, n, t.coef); break;
      case R5_Q: lw.add(Qc, qlen, t.coef); break;
      case R5_F: lw.add(Fc[t.idx], n, t.coef); break;
      case R5_T: lw.add(Tc[t.idx], n, t.coef); break;
      case R5_SELF: lw.add(sFc, n, t.coef); break;
      case R5_SELT: lw.add(sTc, n, t.coef); break;
      case R5_POLT: lw.add(polT, n, t.coef); break;
    }
  }
  lw.c0 = r5.c0;
  const Fr one = Fr::one();
  uint32_t* Pbuf;
  uint64_t L;
  L = qlen > n ? qlen : n;
  Pbuf = c.buf("Pw", 32 * L);
  uint32_t* Wx = c.buf("Wxi", 32 * L);
  const uint32_t* xp1 = xpowers(c, xi);
  const uint32_t* xp2 = xpowers(c, xiw);
  // two lanes: W_x's linear combination and division on lane 0 while W_xw's run on lane 1 (and its
  // commitment starts there right after); the commitments balance as W_x[0, h) on lane 0 and W_xw +
  // W_x[h, L - 1) on lane 1, h = half of all their points
  fork_lanes(c);
  run_lincomb(c.st, Pbuf, L, lw);
  const uint32_t dtiles = (uint32_t)((L + EVAL_TILE - 1) / EVAL_TILE);
  launch_divide(c.st, Wx, flags + 2, Pbuf, L, xp1, c.buf("div_part", 32 * (dtiles + 1)),
                c.buf("div_carry", 32 * (dtiles + 1)));
  // W_{xi w} = (S - S(xi w)) / (X - xi w)
  LcTerms l2;
  l2.add(Sc, n, one);
  l2.c0 = sxiw.neg();
  uint32_t* P2 = c.buf("Pw2", E);
  uint32_t* Wxw = c.buf("Wxiw", E);
  run_lincomb(s2, P2, n, l2);
  launch_divide(s2, Wxw, flags + 3, P2, n, xp2, c.buf("div_part2", 32 * (ntiles + 1)),
                c.buf("div_carry2", 32 * (ntiles + 1)));
  check_launch();
  Commit cW2 = commit_launch(c, Wxw, n - 1, slot++, 1);
  lane_join(c, c.st, s2);  // W_x[h, L - 1) on lane 1 needs W_x
  Commit cW1 = commit_launch_split(c, Wx, L - 1, (L - 1 + n - 1) / 2, slot);
  slot += 2;
  HC(hipMemcpyAsync(h_flags, flags, 64, hipMemcpyDeviceToHost, c.st));
  c.sync();
  if (h_flags[2] || h_flags[3]) throw KgsError(KGS_E_DOES_NOT_DIVIDE, "Polynomial does not divide");
  commits_finish(c, {cW1, cW2}, {com[ci].data(), com[ci + 1].data()});
  ci += 2;
  lap(4);

  for (int i = 0; i < ncom; i++) memcpy(com_out + 64 * i, com[i].data(), 64);
  for (size_t i = 0; i < evals.size(); i++) evals[i].to_bytes(ev_out + 32 * i);
  c.reset_staging();
}


// ------------------------------------------------------------------ host G2 (synthetic ptau): host_pairing.hpp
using host::Fq2;
using host::G2A;
using host::g2_add;
using host::g2_gen;
using host::g2_lem;

// fixed-base table (d * 2^(8j)) G, affine LEM, 32 x 256
std::vector<uint8_t> g1_fixed_table() {
  std::vector<uint8_t> tbl(32 * 256 * 64, 0);
  uint8_t gen[64];
  Fq::one().to_bytes(gen);
  Fq::from_u64(2).to_bytes(gen + 32);
  host::G1 base = host::G1::from_affine_lem(gen);
  for (int j = 0; j < 32; j++) {
    host::G1 acc = host::G1::inf();
    for (int d = 1; d < 256; d++) {
      acc = acc.add(base);
      acc.to_affine_lem(&tbl[64 * (j * 256 + d)]);
    }
    for (int s = 0; s < 8; s++) base = base.dbl();
  }
  return tbl;
}

}  // namespace

// ================================================================== C-ABI
extern "C" {


int kgs_ctx_create(int device, kgs_ctx_t** out) {
  try {
    if (!out) throw KgsError(KGS_E_ARG, "out is NULL");
    int ndev = 0;
    HC(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) throw KgsError(KGS_E_ARG, "no such HIP device");
    HC(hipSetDevice(device));
    auto* c = new kgs_ctx();
    c->device = device;
    HC(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    // the second MSM lane and the copy stream are created on first use: contexts that never need
    // them keep one stream (several in-flight contexts share the device's few hardware queues)
    c->d_scal = c->buf("scalars", kgs_ctx::SCAL_BYTES);
    // reference-identical behaviour on degenerate inputs by default (kgs.h); KGS_REFERENCE_QUIRKS=0
    // selects the exact-math prover
    c->ref_quirks = true;
    if (const char* e = getenv("KGS_REFERENCE_QUIRKS")) c->ref_quirks = e[0] != '0';
    c->ensure_pin(8 << 20);
    *out = c;
    return KGS_OK;
  } catch (const KgsError& e) {
    return kgs_fail(e);
  } catch (const std::exception& e) {
    kgs_errbuf() = e.what();
    return KGS_E_HIP;
  }
}

void kgs_ctx_destroy(kgs_ctx_t* ctx) {
  if (!ctx) return;
  { std::lock_guard<std::mutex> lk(ctx->mu); }  // wait for a call still running on another thread
  delete ctx;
}

#define CTX_LOCK(c) std::lock_guard<std::mutex> ctx_lock_(c->mu)
#define API_BEGIN try {
#define API_END                               \
  }                                           \
  catch (const KgsError& e) {                 \
    return kgs_fail(e);                           \
  }                                           \
  catch (const std::exception& e) {           \
    kgs_errbuf() = e.what();                         \
    return KGS_E_HIP;                         \
  }                                           \
  return KGS_OK;

int kgs_device_count(int* count) {
  API_BEGIN
  if (!count) throw KgsError(KGS_E_ARG, "NULL argument");
  int n = 0;
  HC(hipGetDeviceCount(&n));
  *count = n;
  API_END
}

int kgs_ctx_set_reference_quirks(kgs_ctx_t* ctx, int on) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  ctx->ref_quirks = on != 0;
  API_END
}

int kgs_srs_load_points(kgs_ctx_t* ctx, const uint8_t* g1_lem, uint64_t npts, int power, int nbits_max) {
  API_BEGIN
  if (!ctx || !g1_lem) throw KgsError(KGS_E_ARG, "NULL argument");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if (nbits_max < 0) nbits_max = power;
  if (nbits_max > 28) throw KgsError(KGS_E_ARG, "nbits_max must be <= 28");
  uint64_t need = 1ull << (nbits_max + 1);
  if (npts < need) need = npts;
  load_points(*ctx, g1_lem, need, power, nbits_max, "");
  API_END
}

}  // extern "C"

// ptau section 2 -> device tables: the first 2^(nbits_max+1) points, or (world > 1) rank's slice of
// them, the points rank + world * j, read in chunks and subsampled on the host
static void load_ptau_impl(kgs_ctx_t* ctx, const char* path, int nbits_max, int rank, int world) {
  if (!ctx || !path) throw KgsError(KGS_E_ARG, "NULL argument");
  if (world < 1 || world > 16 || (world & (world - 1)) || rank < 0 || rank >= world)
    throw KgsError(KGS_E_ARG, "SRS slice: world must be 1, 2, 4, 8 or 16 and 0 <= rank < world");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  FILE* f = fopen(path, "rb");
  if (!f) throw KgsError(KGS_E_IO, std::string("cannot open ") + path);
  std::unique_ptr<FILE, int (*)(FILE*)> guard(f, fclose);
  PtauInfo info = read_ptau_header(f, path);
  if (nbits_max < 0 || nbits_max > info.power) nbits_max = info.power;
  if (nbits_max > 28) throw KgsError(KGS_E_SRS, "ptau power above 28 is not supported");
  // file identity: the reference re-reads the file on every call, so a rewritten file (same path,
  // new size or mtime) must not hit the device cache
  struct stat stt;
  if (fstat(fileno(f), &stt) != 0) throw KgsError(KGS_E_IO, std::string("cannot stat ") + path);
  char real[4096];
  const char* rp = realpath(path, real) ? real : path;
  const std::string file = std::string(rp) + "#" + std::to_string((long long)stt.st_size) + "#" +
                           std::to_string((long long)stt.st_mtim.tv_sec) + "." + std::to_string((long long)stt.st_mtim.tv_nsec);
  // grow-only: tables loaded for a larger domain of the same file (and slice) serve every smaller proof
  if (ctx->srs && ctx->srs->file == file && ctx->srs->nbits_max >= nbits_max && ctx->srs->slice_rank == rank &&
      ctx->srs->slice_world == world)
    return;
  uint64_t avail = info.s2_size / 64;
  if (avail < 2) throw KgsError(KGS_E_IO, std::string(path) + ": ptau has no tauG1 section");
  uint64_t need = 1ull << (nbits_max + 1);
  if (need > avail) need = avail;
  const uint64_t mine = need > (uint64_t)rank ? (need - rank + world - 1) / world : 0;  // points rank + world j < need
  if (mine < 2) throw KgsError(KGS_E_ARG, "SRS slice needs at least 2 points");
  std::vector<uint8_t> pts(mine * 64);
  if (fseeko(f, (off_t)info.s2_pos, SEEK_SET)) throw KgsError(KGS_E_IO, "cannot read tauG1 section");
  if (world == 1) {
    if (fread(pts.data(), 1, pts.size(), f) != pts.size()) throw KgsError(KGS_E_IO, "cannot read tauG1 section");
  } else {
    const uint64_t CH = (uint64_t)world << 16;  // points per read
    std::vector<uint8_t> buf(CH * 64);
    uint64_t j = 0;
    for (uint64_t p0 = 0; p0 < need; p0 += CH) {
      const uint64_t cnt = need - p0 < CH ? need - p0 : CH;
      if (fread(buf.data(), 1, cnt * 64, f) != cnt * 64) throw KgsError(KGS_E_IO, "cannot read tauG1 section");
      for (uint64_t q = (uint64_t)rank; q < cnt; q += world) memcpy(&pts[64 * j++], &buf[64 * q], 64);
    }
  }
  load_points(*ctx, pts.data(), mine, info.power, nbits_max, file, rank, world);
}

extern "C" {

int kgs_srs_load_ptau(kgs_ctx_t* ctx, const char* path, int nbits_max) {
  API_BEGIN
  load_ptau_impl(ctx, path, nbits_max, 0, 1);
  API_END
}

int kgs_srs_load_ptau_slice(kgs_ctx_t* ctx, const char* path, int nbits_max, int rank, int world) {
  API_BEGIN
  load_ptau_impl(ctx, path, nbits_max, rank, world);
  API_END
}

int kgs_srs_slice_info(kgs_ctx_t* ctx, int* rank, int* world, uint64_t* table_bytes) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  if (rank) *rank = ctx->srs_slice_rank;
  if (world) *world = ctx->srs_slice_world;
  if (table_bytes) *table_bytes = ctx->srs ? (uint64_t)ctx->tb.W * ctx->tb.npts * 64 : 0;
  API_END
}

int kgs_srs_info(kgs_ctx_t* ctx, int* power, uint64_t* npts, int* window_c) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  if (power) *power = ctx->srs_power;
  if (npts) *npts = ctx->tb.npts;
  if (window_c) *window_c = ctx->tb.c;
  API_END
}

int kgs_ptau_write_synthetic(kgs_ctx_t* ctx, const char* path, int power, const uint8_t tau_std[32]) {
  API_BEGIN
  if (!path || !tau_std || power < 1 || power > 28) throw KgsError(KGS_E_ARG, "bad argument");
  uint64_t s[4];
  memcpy(s, tau_std, 32);
  Fr tau = Fr::from_std(s);
  const uint64_t n1 = (1ull << (power + 1)) - 1;
  std::vector<uint8_t> g1(n1 * 64);
  std::vector<uint8_t> tbl = g1_fixed_table();
  if (ctx) {
    CTX_LOCK(ctx);
    HC(hipSetDevice(ctx->device));
    ctx->reset_staging();
    uint32_t* d_tau = ctx->scal(&tau, 1);
    uint32_t* pw = ctx->buf("syn_pow", 32 * n1);
    uint32_t* xy = ctx->buf("syn_xyzz", 128 * n1);
    uint32_t* scr = ctx->buf("syn_scr", 32 * n1);
    uint32_t* aff = ctx->buf("syn_aff", 64 * n1);
    uint32_t* dtbl = ctx->buf("syn_tbl", tbl.size());
    HC(hipMemcpyAsync(dtbl, tbl.data(), tbl.size(), hipMemcpyHostToDevice, ctx->st));
    launch_powers(ctx->st, pw, n1, d_tau, nullptr);
    launch_fixed_base(ctx->st, xy, pw, n1, dtbl);
    launch_batch_affine(ctx->st, aff, xy, scr, n1);
    check_launch();
    HC(hipMemcpyAsync(g1.data(), aff, g1.size(), hipMemcpyDeviceToHost, ctx->st));
    ctx->reset_staging();
  } else {
    Fr t = Fr::one();
    for (uint64_t i = 0; i < n1; i++) {
      uint64_t e[4];
      t.to_std(e);
      host::G1 acc = host::G1::inf();
      for (int j = 0; j < 32; j++) {
        unsigned d = (unsigned)((e[j >> 3] >> (8 * (j & 7))) & 0xff);
        if (d) acc = acc.add(host::G1::from_affine_lem(&tbl[64 * (j * 256 + d)]));
      }
      acc.to_affine_lem(&g1[64 * i]);
      t = t * tau;
    }
  }
  // [1]_2, [tau]_2
  G2A g = g2_gen(), acc{g.x, g.y, true}, base = g;
  uint64_t e[4];
  tau.to_std(e);
  for (int i = 0; i < 256; i++) {
    if ((e[i >> 6] >> (i & 63)) & 1) acc = g2_add(acc, base);
    base = g2_add(base, base);
  }
  uint8_t g2[256];
  g2_lem(g, g2);
  g2_lem(acc, g2 + 128);
  FILE* f = fopen(path, "wb");
  if (!f) throw KgsError(KGS_E_IO, std::string("cannot create ") + path);
  std::unique_ptr<FILE, int (*)(FILE*)> guard(f, fclose);
  auto w32 = [&](uint32_t x) { fwrite(&x, 4, 1, f); };
  auto w64 = [&](uint64_t x) { fwrite(&x, 8, 1, f); };
  fwrite("ptau", 1, 4, f);
  w32(1);
  w32(3);
  w32(1);
  w64(44);
  w32(32);
  fwrite(host::FQ_MOD.p, 1, 32, f);
  w32((uint32_t)power);
  w32((uint32_t)power);
  w32(2);
  w64(g1.size());
  fwrite(g1.data(), 1, g1.size(), f);
  w32(3);
  w64(256);
  if (fwrite(g2, 1, 256, f) != 256) throw KgsError(KGS_E_IO, "write failed");
  API_END
}


}  // extern "C"

namespace kgsi {
// host copies between pageable caller buffers and the pinned staging area, split over threads; the
// 16 threads (a GPU's host share) are divided among the contexts copying at the same time, so that
// several proofs in flight through the host-buffer boundary do not oversubscribe the cores. The
// helpers are a persistent pool (spawning 8-16 threads per call cost ~0.1 ms, paid several times per
// proof once inputs are fed in pieces); the calling thread copies too, so a busy pool never stalls it.
static std::atomic<int> g_copy_active{0};
// host threads for the staging copies of all contexts together (KGS_COPY_THREADS, default 16: a GPU's
// share of the host's cores)
static unsigned copy_threads() {
  static const unsigned n = [] {
    const char* e = getenv("KGS_COPY_THREADS");
    const int v = e ? atoi(e) : 16;
    return (unsigned)(v >= 1 && v <= 64 ? v : 16);
  }();
  return n;
}
namespace {
// The staging copy's stores: cached (memcpy) or 16 B non-temporal. NT stores bypass the caches and
// copy a 32 MiB vector into pinned staging in 0.26 ms with 4 threads against 0.44 ms for memcpy
// (profiles/ubench/host_copy_bw.cpp, profiles/r06/host_copy_bw.txt), but then the H2D DMA reads the
// staging from DRAM instead of the host's L3, and F's DMA, not its copy, is what a lone proof waits
// for. Measured (same boxes, interleaved): a lone proof through the JavaScript module is faster with
// cached stores, median 15.1-16.1 vs 16.8-17.8 ms (4 x 15 samples, profiles/r06/js_lat_ab.txt; again
// 15.7-16.6 vs 16.9-17.9, profiles/r06/copy_final_ab/). Four proofs in flight are faster with NT
// stores, 0.9727 vs 0.9664 of device-resident (12 samples each, profiles/r06/inflight_store_ab/). So by
// default (KGS_COPY_NT unset) a copy uses NT stores when another proof of the process is in progress,
// cached stores when its proof is alone; KGS_COPY_NT=0 / 1 forces one kind. With NT stores the sfence
// makes the lines globally visible before the piece is counted done, i.e. before its DMA is enqueued.
std::atomic<int> g_proofs_active{0};  // kgs_prove calls in progress in the process
bool copy_nt_now() {
  static const int mode = [] {
    const char* e = getenv("KGS_COPY_NT");
    return e && e[0] == '1' ? 1 : e && e[0] == '0' ? 0 : -1;
  }();
  return mode == 1 || (mode < 0 && g_proofs_active.load(std::memory_order_relaxed) > 1);
}
void copy_stores(uint8_t* d, const uint8_t* s, size_t n, bool nt) {
  if (!nt) {
    memcpy(d, s, n);
    return;
  }
  size_t i = 0;
  const size_t head = (16 - ((uintptr_t)d & 15)) & 15;
  if (head) {
    const size_t h = std::min(head, n);
    memcpy(d, s, h);
    i = h;
  }
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128((const __m128i*)(s + i)), b = _mm_loadu_si128((const __m128i*)(s + i + 16));
    const __m128i c = _mm_loadu_si128((const __m128i*)(s + i + 32)), e = _mm_loadu_si128((const __m128i*)(s + i + 48));
    _mm_stream_si128((__m128i*)(d + i), a);
    _mm_stream_si128((__m128i*)(d + i + 16), b);
    _mm_stream_si128((__m128i*)(d + i + 32), c);
    _mm_stream_si128((__m128i*)(d + i + 48), e);
  }
  if (i < n) memcpy(d + i, s + i, n - i);
  _mm_sfence();
}

// Invariants (DESIGN.md §13 "The round-5 illegal-address fault"): a piece is claimed exactly once,
// before par_copy / stream_copy returns, and pool threads make no HIP call (every DMA is enqueued by
// the thread that owns the call). Queue entries outlive their task (a helper that wakes late pops a
// finished task): such a late `work()` must claim nothing, which `closed` checks.
struct CopyTask {
  std::vector<CopyJob> pieces;
  std::atomic<size_t> next{0}, done{0};
  std::atomic<bool> closed{false};  // set once the owner has seen every piece done
  // stream_copy: pieces left to copy per DMA piece (piece i belongs to DMA piece i / per_dma)
  std::unique_ptr<std::atomic<uint32_t>[]> left;
  size_t per_dma = 0;
  bool nt = false;  // non-temporal stores (decided once per copy: copy_nt_now)
  std::mutex mu;
  std::condition_variable cv;
  bool copy_one(size_t i) {  // false: nothing left to claim
    if (i >= pieces.size()) return false;
    if (closed.load(std::memory_order_acquire)) {
      fprintf(stderr, "kgs: copy piece %zu claimed after its task completed\n", i);
      abort();
    }
    copy_stores(pieces[i].dst, pieces[i].src, pieces[i].len, nt);
    if (left) left[i / per_dma].fetch_sub(1, std::memory_order_release);
    return true;
  }
  void work() {
    size_t mine = 0;
    while (copy_one(next.fetch_add(1))) mine++;
    if (mine && done.fetch_add(mine) + mine == pieces.size()) {
      std::lock_guard<std::mutex> lk(mu);
      cv.notify_all();
    }
  }
};
struct CopyPool {  // leaked on purpose: its detached threads outlive static destruction
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::shared_ptr<CopyTask>> q;
  explicit CopyPool(unsigned n) {
    for (unsigned t = 0; t < n; t++)
      std::thread([this] {
        for (;;) {
          std::shared_ptr<CopyTask> task;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return !q.empty(); });
            task = std::move(q.back());
            q.pop_back();
          }
          task->work();
        }
      }).detach();
  }
  static CopyPool& get() {
    static CopyPool* p = new CopyPool(copy_threads());
    return *p;
  }
};
struct Active {  // copies running at once in the process: they share the copy threads
  int n;
  Active() : n(g_copy_active.fetch_add(1) + 1) {}
  ~Active() { g_copy_active.fetch_sub(1); }
};
// threads (this one included) for one copy: KGS_COPY_TASK_THREADS (default 2), within the share of
// the copy threads left by the other copies running. The host copy bandwidth of the GPU box peaks at
// 2-4 threads (profiles/r06/host_copy_bw.txt), but the proof does not get faster with it: F_0's DMA,
// not its copy, sets its arrival. Same-box A/Bs (profiles/r06/copy_ab*, f0_ab): single-proof median
// 14.43 ms with 2 threads, 14.82 with 4, 14.54 for round 5's span-by-span copy; in flight all within
// the run-to-run spread (87.7-90.8 proofs/s against 92.7-93.1 device-resident)
unsigned task_threads(const Active& a, size_t pieces) {
  static const unsigned per = [] {
    const char* e = getenv("KGS_COPY_TASK_THREADS");
    const int v = e ? atoi(e) : 2;
    return (unsigned)(v >= 1 && v <= 64 ? v : 2);
  }();
  unsigned nth = std::min(per, std::max(1u, copy_threads() / (unsigned)std::max(1, a.n)));
  return std::max(1u, std::min<unsigned>(nth, (unsigned)pieces));
}
void start_helpers(const std::shared_ptr<CopyTask>& task, unsigned nth) {
  if (nth <= 1) return;
  CopyPool& pool = CopyPool::get();
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    for (unsigned t = 1; t < nth; t++) pool.q.push_back(task);  // helpers; the calling thread is the nth
  }
  pool.cv.notify_all();
}
}  // namespace

void par_copy(const std::vector<CopyJob>& jobs) {
  const size_t piece = 1u << 20;
  auto task = std::make_shared<CopyTask>();
  task->nt = copy_nt_now();
  for (const auto& j : jobs)
    for (size_t o = 0; o < j.len; o += piece) task->pieces.push_back({j.dst + o, j.src + o, std::min(piece, j.len - o)});
  Active active;
  start_helpers(task, task_threads(active, task->pieces.size()));
  task->work();
  std::unique_lock<std::mutex> lk(task->mu);
  task->cv.wait(lk, [&] { return task->done.load() == task->pieces.size(); });
  task->closed.store(true, std::memory_order_release);
}

// One vector into pinned staging, copied in 256 KiB pieces claimed in address order by this thread
// and the pool's helpers; `ready(offset, len)` runs on THIS thread for each `dma`-byte span, in order,
// as soon as every piece of it is copied (it enqueues that span's DMA). So the first DMA starts after
// one span's copy and the link is fed while the rest is still being copied, at the copy bandwidth of
// several threads (round 5 copied span by span with two threads each, ~1.2 ms for a 32 MiB vector).
// An exception from `ready` is held until every piece is copied (helpers never outlive the call's
// writes into the staging), then rethrown; later spans are not enqueued.
void stream_copy(uint8_t* dst, const uint8_t* src, size_t len, size_t dma, const std::function<void(size_t, size_t)>& ready) {
  const size_t sub = (size_t)256 << 10;
  dma = std::max(sub, dma / sub * sub);
  auto task = std::make_shared<CopyTask>();
  task->nt = copy_nt_now();
  for (size_t o = 0; o < len; o += sub) task->pieces.push_back({dst + o, src + o, std::min(sub, len - o)});
  const size_t ndma = (len + dma - 1) / dma;
  task->per_dma = dma / sub;
  task->left.reset(new std::atomic<uint32_t>[ndma]);
  for (size_t k = 0; k < ndma; k++)
    task->left[k].store((uint32_t)std::min(task->per_dma, task->pieces.size() - k * task->per_dma));
  Active active;
  start_helpers(task, task_threads(active, task->pieces.size()));
  size_t issued = 0, mine = 0;
  std::exception_ptr err;
  auto flush = [&] {
    while (issued < ndma && task->left[issued].load(std::memory_order_acquire) == 0) {
      const size_t o = issued * dma;
      if (!err) {
        try {
          ready(o, std::min(dma, len - o));
        } catch (...) {
          err = std::current_exception();
        }
      }
      issued++;
    }
  };
  while (task->copy_one(task->next.fetch_add(1))) {
    mine++;
    flush();
  }
  if (mine) task->done.fetch_add(mine);
  while (issued < ndma) {  // the helpers' last pieces (each at most one 256 KiB copy away)
    flush();
    if (issued < ndma) _mm_pause();
  }
  task->closed.store(true, std::memory_order_release);
  if (err) std::rethrow_exception(err);
}

// Caller buffers the DMAs can read / write in place: memory the caller already pinned (hipHostMalloc,
// kgs_host_register) is used as it is and left alone, so a caller that keeps its buffers across
// proofs skips the staging copy. Registering pageable buffers per call (KGS_HOST_REGISTER=1) is kept
// as an opt-in only: measured at 2^20 it makes the host path slower, 21.5 vs 16.0 ms per proof, and
// the JS concurrent rate 44.9 vs 78.8 proofs/s (register + unregister of 2 x 32 MiB costs more than
// the ~1 ms copy it saves, and registrations serialise across contexts), profiles/r03/boundary_ab.txt.
// Per-call registrations are released after every stream of the context is drained (also on an error
// path). Concurrent calls may pass the same buffer (e.g. one selector vector shared by several
// proofs): the registrations are reference-counted process-wide, so the first call to finish does not
// unpin memory another call is still DMA-ing. Overlapping buffers with different starts fail to
// register and take the staging path.
// Drains every stream of the context when the call it guards leaves by an exception. Rank-group
// contexts are left alone: their main stream may wait in an exchange whose peers failed (the group's
// abort releases it), and they never DMA caller memory in place.
struct DrainOnError {
  kgs_ctx* ctx;
  int unwinding = std::uncaught_exceptions();
  explicit DrainOnError(kgs_ctx* c) : ctx(c) {}
  ~DrainOnError() {
    if (std::uncaught_exceptions() <= unwinding || ctx->group) return;
    hipSetDevice(ctx->device);
    for (hipStream_t s : {ctx->st, ctx->st2, ctx->st_copy, ctx->st_wb})
      if (s) (void)hipStreamSynchronize(s);
    (void)hipGetLastError();
  }
};

static std::mutex g_pin_mu;
static std::map<void*, std::pair<size_t, int>> g_pins;  // start -> (bytes, calls holding it)
struct HostPins {
  kgs_ctx* ctx;
  std::vector<void*> mine;
  explicit HostPins(kgs_ctx* c) : ctx(c) {}
  static bool pinned_elsewhere(const void* p) {
    hipPointerAttribute_t a{};
    const bool ok = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // a pageable pointer is an error here: not a sticky launch error
    return ok;
  }
  bool pin(const void* cp, size_t n) {
    void* p = const_cast<void*>(cp);
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.find(p);
    if (it != g_pins.end()) {
      if (it->second.first < n) return false;
      it->second.second++;
      mine.push_back(p);
      return true;
    }
    if (pinned_elsewhere(p)) return true;  // the caller's own pinned memory: use, never unpin
    static const bool reg = getenv("KGS_HOST_REGISTER") != nullptr;  // opt-in, see above
    if (!reg) return false;
    if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    g_pins[p] = {n, 1};
    mine.push_back(p);
    return true;
  }
  static void drop(void* p) {  // under g_pin_mu
    auto it = g_pins.find(p);
    if (it != g_pins.end() && --it->second.second == 0) {
      hipHostUnregister(p);
      g_pins.erase(it);
    }
  }
  void release_from(size_t k) {  // the pins made after the first k (no DMA issued on them yet)
    std::lock_guard<std::mutex> lk(g_pin_mu);
    while (mine.size() > k) {
      drop(mine.back());
      mine.pop_back();
    }
  }
  ~HostPins() {
    if (mine.empty()) return;
    hipSetDevice(ctx->device);
    if (ctx->st) hipStreamSynchronize(ctx->st);
    if (ctx->st2) hipStreamSynchronize(ctx->st2);
    if (ctx->st_copy) hipStreamSynchronize(ctx->st_copy);
    if (ctx->st_wb) hipStreamSynchronize(ctx->st_wb);
    std::lock_guard<std::mutex> lk(g_pin_mu);
    for (void* p : mine) drop(p);
  }
};
}  // namespace kgsi

extern "C" {

int kgs_host_register(void* ptr, uint64_t bytes) {
  API_BEGIN
  if (!ptr || !bytes) throw KgsError(KGS_E_ARG, "NULL argument");
  HC(hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault));
  API_END
}

int kgs_host_unregister(void* ptr) {
  API_BEGIN
  if (!ptr) throw KgsError(KGS_E_ARG, "NULL argument");
  HC(hipHostUnregister(ptr));
  API_END
}

int kgs_test_stream_copy(uint8_t* dst, const uint8_t* src, uint64_t len, uint64_t span, int fail_at,
                         uint64_t* spans_out, int max, int* nspans) {
  API_BEGIN
  if (!dst || !src || !nspans || (max > 0 && !spans_out)) throw KgsError(KGS_E_ARG, "NULL argument");
  *nspans = 0;
  stream_copy(dst, src, (size_t)len, (size_t)span, [&](size_t o, size_t) {
    if (*nspans == fail_at) throw KgsError(KGS_E_HIP, "injected span failure");
    if (*nspans < max) spans_out[*nspans] = o;
    (*nspans)++;
  });
  API_END
}

int kgs_ctx_idle(kgs_ctx_t* ctx) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  for (hipStream_t s : {ctx->st, ctx->st2, ctx->st_copy, ctx->st_wb}) {
    if (!s) continue;
    const hipError_t e = hipStreamQuery(s);
    if (e == hipErrorNotReady) return 0;
    HC(e);
  }
  return 1;
  API_END
}

int kgs_prove(kgs_ctx_t* ctx, int kind, int nbits, int npols, const uint8_t* const* evals_f,
              const uint8_t* const* evals_t, const uint8_t* sel_f, const uint8_t* sel_t, uint8_t* const* mont_f,
              uint8_t* const* mont_t, uint8_t* commitments_out, uint8_t* evaluations_out) {
  API_BEGIN
  if (!ctx || !evals_f || !evals_t || !commitments_out || !evaluations_out) throw KgsError(KGS_E_ARG, "NULL argument");
  CTX_LOCK(ctx);
  if ((sel_f == nullptr) != (sel_t == nullptr)) throw KgsError(KGS_E_ARG, "selectors must be both given or both NULL");
  if (npols < 1 || npols > KGS_MAX_POLS || nbits < 1 || nbits > 28) throw KgsError(KGS_E_ARG, "bad shape");
  HC(hipSetDevice(ctx->device));
  // declared first, so destroyed last (after the feeder and the write-back thread are joined): an
  // error return drains the context's streams, so no DMA of this call still reads or writes caller
  // memory (pinned inputs DMA'd in place, pinned write-back targets) once the caller has it back
  DrainOnError drain(ctx);
  struct ProofActive {  // kgs_prove calls in progress (the staging copy's store choice, copy_nt_now)
    ProofActive() { g_proofs_active.fetch_add(1, std::memory_order_relaxed); }
    ~ProofActive() { g_proofs_active.fetch_sub(1, std::memory_order_relaxed); }
  } proof_active;
  const uint64_t n = 1ull << nbits;
  const size_t E = 32 * n;
  ProveIn in;
  in.kind = kind;
  in.nbits = nbits;
  in.npols = npols;
  // pageable caller buffers -> write-combined pinned staging (parallel host copies) -> DMAs; the
  // Montgomery write-back goes device -> its own pinned slots (st_wb) -> caller (a host thread)
  const int nvec = 2 * npols + (sel_f ? 2 : 0);
  uint8_t* pin_in = ctx->io_in((size_t)nvec * E);
  const bool any_wb = mont_f || mont_t;
  uint8_t* pio = any_wb ? ctx->io((size_t)2 * npols * E) : nullptr;  // write-back slots
  std::vector<CopyJob> in_jobs;
  for (int i = 0; i < npols; i++) {
    in_jobs.push_back({pin_in + (size_t)(2 * i) * E, evals_f[i], E});
    in_jobs.push_back({pin_in + (size_t)(2 * i + 1) * E, evals_t[i], E});
  }
  if (sel_f) {
    in_jobs.push_back({pin_in + (size_t)(2 * npols) * E, sel_f, E});
    in_jobs.push_back({pin_in + (size_t)(2 * npols + 1) * E, sel_t, E});
  }
  ctx->sync();  // the staging area may still feed a previous call's copies
  // inputs: one parallel host copy into the pinned slots, then one DMA per vector
  std::vector<uint32_t*> dsts;
  for (int i = 0; i < npols; i++) {
    dsts.push_back(ctx->buf("in_f" + std::to_string(i), E));
    dsts.push_back(ctx->buf("in_t" + std::to_string(i), E));
  }
  if (sel_f) {
    dsts.push_back(ctx->buf("in_sf", E));
    dsts.push_back(ctx->buf("in_st", E));
  }
  using hclk = std::chrono::steady_clock;
  const auto h0 = hclk::now();
  // each vector in pieces: the host copy of piece p + 1 into the pinned slot runs while piece p is
  // DMA'd, so a vector's DMA ends one piece after its host copy instead of a whole vector after.
  // Vector 0 (F_0, whose transform starts round 1) in 2 MiB pieces, so that its first DMA starts
  // ~0.03 ms into the call and its last ends ~0.04 ms after its copy; the others in 8 MiB pieces
  // (fewer DMA submissions on the feeder thread)
  static const bool span_copy = [] {  // KGS_STREAM_COPY=0: round 5's span-by-span copy (A/B)
    const char* e = getenv("KGS_STREAM_COPY");
    return e && e[0] == '0';
  }();
  auto feed = [&](size_t v, hipStream_t st) {
    static const size_t f0_span = [] {  // KGS_F0_SPAN_MB: DMA span of vector 0 (A/B; default 2 MiB)
      const char* e = getenv("KGS_F0_SPAN_MB");
      const int v = e ? atoi(e) : 2;
      return (size_t)(v >= 1 && v <= 64 ? v : 2) << 20;
    }();
    const size_t span = v == 0 ? f0_span : (size_t)8 << 20;
    if (span_copy) {
      for (size_t o = 0; o < E; o += span) {
        const size_t len = std::min(span, E - o);
        par_copy({{in_jobs[v].dst + o, in_jobs[v].src + o, len}});
        HC(hipMemcpyAsync((uint8_t*)dsts[v] + o, in_jobs[v].dst + o, len, hipMemcpyHostToDevice, st));
      }
      return;
    }
    stream_copy(in_jobs[v].dst, in_jobs[v].src, E, span, [&](size_t o, size_t len) {
      HC(hipMemcpyAsync((uint8_t*)dsts[v] + o, in_jobs[v].dst + o, len, hipMemcpyHostToDevice, st));
    });
  };
  // declared before the feeder: destroyed after it is joined, so streams are drained and buffers
  // unpinned only once nothing can enqueue another DMA on them
  HostPins pins(ctx);
  struct Feeder {  // the input-copy thread of vectors 1.. (joined on every exit path)
    std::thread t;
    std::mutex mu;
    std::condition_variable cv;
    size_t issued = 1;
    std::exception_ptr err;
    ~Feeder() {
      if (t.joinable()) t.join();
    }
  } feeder;
  Range rin("kgs.host.input_copy");
  bool direct = !ctx->group;
  for (size_t v = 0; direct && v < in_jobs.size(); v++) direct = pins.pin(in_jobs[v].src, E);
  if (!direct) pins.release_from(0);
  if (direct) {
    // zero-copy: every input DMA'd straight from the caller's pinned buffer, one after the other on the
    // copy stream (not two streams at once: F_0 then arrives after one vector's transfer time instead
    // of sharing the link with T_0), each with the event its first kernel waits for
    if (!ctx->st_copy) ctx->st_copy = copy_stream();
    while (ctx->ev_in.size() < in_jobs.size()) {
      hipEvent_t e;
      HC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ctx->ev_in.push_back(e);
    }
    in.ready.assign(in_jobs.size(), nullptr);
    for (size_t v = 0; v < in_jobs.size(); v++) {
      HC(hipMemcpyAsync(dsts[v], in_jobs[v].src, E, hipMemcpyHostToDevice, ctx->st_copy));
      HC(hipEventRecord(ctx->ev_in[v], ctx->st_copy));
      in.ready[v] = ctx->ev_in[v];
    }
  } else if (ctx->group) {  // the distributed prover reads every input at once
    par_copy(in_jobs);
    for (size_t v = 0; v < in_jobs.size(); v++)
      HC(hipMemcpyAsync(dsts[v], in_jobs[v].dst, E, hipMemcpyHostToDevice, ctx->st));
  } else {
    // pipelined: vector v's host copy into its pinned slot overlaps vector v - 1's DMA; vector 0
    // goes on the main stream, the others on the copy stream with an event that the main stream
    // waits for right before the vector's first kernel, so F_0's transform starts while the rest
    // are still in flight. (The Montgomery write-back has pinned slots of its own, written on st_wb:
    // vector v's D2H is ordered after its conversion kernel, which waits on ev_in[v], i.e. after
    // vector v's input DMA.)
    if (!ctx->st_copy) ctx->st_copy = copy_stream();
    while (ctx->ev_in.size() < in_jobs.size()) {
      hipEvent_t e;
      HC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ctx->ev_in.push_back(e);
    }
    in.ready.assign(in_jobs.size(), nullptr);
    // KGS_F0_STREAM=copy (A/B): F_0's DMAs on the copy stream too, the main stream waits on ev_in[0]
    static const bool f0_on_copy = [] {
      const char* e = getenv("KGS_F0_STREAM");
      return e && !strcmp(e, "copy");
    }();
    if (f0_on_copy) {
      feed(0, ctx->st_copy);
      HC(hipEventRecord(ctx->ev_in[0], ctx->st_copy));
      in.ready[0] = ctx->ev_in[0];
    } else {
      feed(0, ctx->st);
    }
    // the link carries F_0 first: the copy stream's DMAs start after F_0's last one (ev_in[0] on the
    // main stream, which holds only F_0's DMAs here). With the multi-threaded staging copy, T_0's DMAs
    // otherwise shared the link with F_0's and F_0 arrived ~0.5 ms later (profiles/r06/copy_ab/);
    // KGS_FEED_ORDER=0 lets them overlap (A/B)
    static const bool ordered = [] {
      const char* e = getenv("KGS_FEED_ORDER");
      return !(e && e[0] == '0');
    }();
    const bool wait_f0 = ordered && in_jobs.size() > 1 && !f0_on_copy;  // (same stream: ordered anyway)
    if (wait_f0) HC(hipEventRecord(ctx->ev_in[0], ctx->st));
    for (size_t v = 1; v < in_jobs.size(); v++) in.ready[v] = ctx->ev_in[v];
    // vectors 1.. are copied into their pinned slots and DMA'd by a feeder thread while the prover
    // already enqueues (and the GPU runs) vector 0's work; prove_impl waits for a vector's DMA to be
    // ENQUEUED (input_issued) before its kernels wait on the vector's event
    if (in_jobs.size() > 1) {
      feeder.t = std::thread([&, dev = ctx->device] {
        try {
          HC(hipSetDevice(dev));
          if (wait_f0) HC(hipStreamWaitEvent(ctx->st_copy, ctx->ev_in[0], 0));
          for (size_t v = 1; v < in_jobs.size(); v++) {
            feed(v, ctx->st_copy);
            HC(hipEventRecord(ctx->ev_in[v], ctx->st_copy));
            std::lock_guard<std::mutex> lk(feeder.mu);
            feeder.issued = v + 1;
            feeder.cv.notify_all();
          }
        } catch (...) {
          std::lock_guard<std::mutex> lk(feeder.mu);
          feeder.err = std::current_exception();
          feeder.issued = in_jobs.size();
          feeder.cv.notify_all();
        }
      });
      in.input_issued = [&](size_t v) {
        std::unique_lock<std::mutex> lk(feeder.mu);
        feeder.cv.wait(lk, [&] { return feeder.issued > v; });
        if (feeder.err) std::rethrow_exception(feeder.err);
      };
    }
  }
  rin.pop();
  const auto h1 = hclk::now();
  // the Montgomery write-back: D2H straight into the caller's buffer once it is pinned (the JS addon
  // keeps its recycled output buffers registered), else into the pinned slot + a host copy
  std::vector<bool> wb_direct(2 * npols, false);
  for (int i = 0; i < npols; i++) {
    in.f_std.push_back(dsts[2 * i]);
    in.t_std.push_back(dsts[2 * i + 1]);
    const bool fd = mont_f && mont_f[i] && !ctx->group && pins.pin(mont_f[i], E);
    const bool td = mont_t && mont_t[i] && !ctx->group && pins.pin(mont_t[i], E);
    wb_direct[2 * i] = fd;
    wb_direct[2 * i + 1] = td;
    in.mont_f_out.push_back(mont_f && mont_f[i] ? (fd ? mont_f[i] : pio + (size_t)(2 * i) * E) : nullptr);
    in.mont_t_out.push_back(mont_t && mont_t[i] ? (td ? mont_t[i] : pio + (size_t)(2 * i + 1) * E) : nullptr);
  }
  if (sel_f) {
    in.sel_f = dsts[2 * npols];
    in.sel_t = dsts[2 * npols + 1];
  }
  // the Montgomery forms are in the pinned slots once round 1 is synchronised: copy them to the
  // caller on a host thread while rounds 2-5 run
  std::vector<CopyJob> out_jobs;
  for (int i = 0; i < npols; i++) {
    if (mont_f && mont_f[i] && !wb_direct[2 * i]) out_jobs.push_back({mont_f[i], pio + (size_t)(2 * i) * E, E});
    if (mont_t && mont_t[i] && !wb_direct[2 * i + 1]) out_jobs.push_back({mont_t[i], pio + (size_t)(2 * i + 1) * E, E});
  }
  struct Joiner {
    std::thread t;
    bool failed = false;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } out_copy;
  if (!out_jobs.empty())
    in.after_round1 = [&] {
      out_copy.t = std::thread([&, dev = ctx->device] {
        // the device -> pinned write-back (st_wb) must be complete before the pinned -> caller copy
        if (hipSetDevice(dev) != hipSuccess || (ctx->st_wb && hipStreamSynchronize(ctx->st_wb) != hipSuccess)) {
          out_copy.failed = true;
          return;
        }
        par_copy(out_jobs);
      });
    };
  const auto h2 = hclk::now();
  prove_impl(*ctx, in, commitments_out, evaluations_out);  // ends synchronised
  const auto h3 = hclk::now();
  Range rout("kgs.host.writeback_wait");
  if (out_copy.t.joinable()) out_copy.t.join();
  if (out_copy.failed) throw KgsError(KGS_E_HIP, "Montgomery write-back: copy stream failed");
  rout.pop();
  const auto h4 = hclk::now();
  // host-boundary phases: [6] input copy into pinned staging, [7] prover, [8] write-back wait
  ctx->timing.resize(9, 0.0);
  ctx->timing[6] = std::chrono::duration<double, std::milli>(h1 - h0).count();
  ctx->timing[7] = std::chrono::duration<double, std::milli>(h3 - h2).count();
  ctx->timing[8] = std::chrono::duration<double, std::milli>(h4 - h3).count();
  API_END
}

int kgs_prove_device(kgs_ctx_t* ctx, int kind, int nbits, int npols, const void* const* d_evals_f,
                     const void* const* d_evals_t, const void* d_sel_f, const void* d_sel_t, uint8_t* commitments_out,
                     uint8_t* evaluations_out) {
  API_BEGIN
  if (!ctx || !d_evals_f || !d_evals_t || !commitments_out || !evaluations_out) throw KgsError(KGS_E_ARG, "NULL argument");
  CTX_LOCK(ctx);
  if ((d_sel_f == nullptr) != (d_sel_t == nullptr)) throw KgsError(KGS_E_ARG, "selectors must be both given or both NULL");
  if (npols < 1 || npols > KGS_MAX_POLS || nbits < 1 || nbits > 28) throw KgsError(KGS_E_ARG, "bad shape");
  HC(hipSetDevice(ctx->device));
  DrainOnError drain(ctx);  // no kernel of a failed call still reads the caller's device buffers
  ProveIn in;
  in.kind = kind;
  in.nbits = nbits;
  in.npols = npols;
  for (int i = 0; i < npols; i++) {
    in.f_std.push_back((const uint32_t*)d_evals_f[i]);
    in.t_std.push_back((const uint32_t*)d_evals_t[i]);
  }
  in.sel_f = (const uint32_t*)d_sel_f;
  in.sel_t = (const uint32_t*)d_sel_t;
  prove_impl(*ctx, in, commitments_out, evaluations_out);
  API_END
}

int kgs_last_timing(kgs_ctx_t* ctx, double* rounds_ms, int max_rounds) {
  if (!ctx || !rounds_ms) return KGS_E_ARG;
  CTX_LOCK(ctx);
  int n = (int)ctx->timing.size() < max_rounds ? (int)ctx->timing.size() : max_rounds;
  for (int i = 0; i < n; i++) rounds_ms[i] = ctx->timing[i];
  return n;
}

int kgs_fr_to_mont(kgs_ctx_t* ctx, const uint8_t* in_std, uint8_t* out_mont, uint64_t n) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  uint32_t* a = ctx->buf("prim_a", 32 * n);
  uint32_t* b = ctx->buf("prim_b", 32 * n);
  HC(hipMemcpyAsync(a, in_std, 32 * n, hipMemcpyHostToDevice, ctx->st));
  launch_to_mont(ctx->st, b, a, n);
  check_launch();
  HC(hipMemcpyAsync(out_mont, b, 32 * n, hipMemcpyDeviceToHost, ctx->st));
  ctx->sync();
  API_END
}

// the shim's elementwise maps (host buffers in and out, one launch on ctx's stream)
static void fr_map(kgs_ctx_t* ctx, const uint8_t* in, uint8_t* out, uint64_t n,
                   void (*launch)(hipStream_t, uint32_t*, const uint32_t*, uint64_t)) {
  if (!ctx || (n && (!in || !out))) throw KgsError(KGS_E_ARG, "NULL argument");
  if (!n) return;
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  uint32_t* a = ctx->buf("prim_a", 32 * n);
  uint32_t* b = ctx->buf("prim_b", 32 * n);
  HC(hipMemcpyAsync(a, in, 32 * n, hipMemcpyHostToDevice, ctx->st));
  launch(ctx->st, b, a, n);
  check_launch();
  HC(hipMemcpyAsync(out, b, 32 * n, hipMemcpyDeviceToHost, ctx->st));
  ctx->sync();
}

int kgs_fr_from_mont(kgs_ctx_t* ctx, const uint8_t* in_mont, uint8_t* out_std, uint64_t n) {
  API_BEGIN
  fr_map(ctx, in_mont, out_std, n, launch_from_mont);
  API_END
}

int kgs_fr_batch_inverse(kgs_ctx_t* ctx, const uint8_t* in_mont, uint8_t* out_mont, uint64_t n) {
  API_BEGIN
  fr_map(ctx, in_mont, out_mont, n, launch_fr_batch_inv);
  API_END
}

int kgs_ntt(kgs_ctx_t* ctx, const uint8_t* in_mont, uint8_t* out_mont, int logm, int inverse) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if (logm < 0 || logm > 28) throw KgsError(KGS_E_ARG, "bad logm");
  if (logm > ctx->logM) ensure_domain(*ctx, logm);
  const uint64_t m = 1ull << logm;
  uint32_t* a = ctx->buf("prim_a", 32 * m);
  uint32_t* b = ctx->buf("prim_b", 32 * m);
  ctx->reset_staging();
  HC(hipMemcpyAsync(a, in_mont, 32 * m, hipMemcpyHostToDevice, ctx->st));
  if (inverse) {
    intt_nat(*ctx, b, a, logm);
  } else {
    ntt_dif(ctx->st, a, a, m, logm, nullptr, ctx->tw_fwd, ctx->logM);
    launch_bitrev_copy(ctx->st, b, a, logm);
  }
  check_launch();
  HC(hipMemcpyAsync(out_mont, b, 32 * m, hipMemcpyDeviceToHost, ctx->st));
  ctx->sync();
  API_END
}

int kgs_msm(kgs_ctx_t* ctx, const uint8_t* scalars_mont, uint64_t n, uint8_t out_lem[64]) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if (n > ctx->tb.npts) throw KgsError(KGS_E_SRS, "MSM larger than the resident SRS");
  ctx->reset_staging();
  uint32_t* a = ctx->buf("prim_a", 32 * (n ? n : 1));
  HC(hipMemcpyAsync(a, scalars_mont, 32 * n, hipMemcpyHostToDevice, ctx->st));
  Commit cm = commit_launch(*ctx, a, n, 0);
  ctx->sync();
  commit_finish(*ctx, cm, out_lem);
  ctx->reset_staging();
  API_END
}

int kgs_ctx_set_shard(kgs_ctx_t* ctx, int rank, int world, kgs_allgather_fn fn, void* user) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "ctx is NULL");
  CTX_LOCK(ctx);
  if (world < 1 || rank < 0 || rank >= world) throw KgsError(KGS_E_ARG, "bad shard rank/world");
  if (world > 1 && !fn) throw KgsError(KGS_E_ARG, "sharding needs an all-gather callback");
  ctx->shard_rank = world > 1 ? rank : 0;
  ctx->shard_world = world;
  ctx->shard_fn = world > 1 ? fn : nullptr;
  ctx->shard_user = world > 1 ? user : nullptr;
  API_END
}

int kgs_ctx_set_msm_lanes(kgs_ctx_t* ctx, int lanes) {
  API_BEGIN
  if (!ctx || lanes < 1 || lanes > 2) throw KgsError(KGS_E_ARG, "msm lanes must be 1 or 2");
  CTX_LOCK(ctx);
  ctx->msm_lanes = lanes;
  API_END
}

int kgs_shard_range(uint64_t n, int rank, int world, uint64_t* lo, uint64_t* hi) {
  API_BEGIN
  if (world < 1 || rank < 0 || rank >= world || !lo || !hi) throw KgsError(KGS_E_ARG, "bad shard rank/world");
  shard_range(n, rank, world, *lo, *hi);
  API_END
}

int kgs_msm_combine(const uint8_t* T_all, int nparts, int c, uint8_t out_lem[64]) {
  API_BEGIN
  if (!T_all || !out_lem || nparts < 1 || c < 1 || c > 32) throw KgsError(KGS_E_ARG, "bad msm_combine arguments");
  combine_partials(T_all, (size_t)c * 128, nparts, c, out_lem);
  API_END
}

int kgs_grand_build(kgs_ctx_t* ctx, int kind, const uint8_t* f_mont, const uint8_t* t_mont, const uint8_t* sel_f,
                    const uint8_t* sel_t, const uint8_t gamma_mont[32], uint64_t n, uint8_t* out_mont) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if ((sel_f == nullptr) != (sel_t == nullptr)) throw KgsError(KGS_E_ARG, "selectors must be both given or both NULL");
  ctx->reset_staging();
  const size_t E = 32 * n;
  uint32_t* f = ctx->buf("gb_f", E);
  uint32_t* t = ctx->buf("gb_t", E);
  uint32_t* o = ctx->buf("gb_o", E);
  uint32_t *sf = nullptr, *st = nullptr;
  HC(hipMemcpyAsync(f, f_mont, E, hipMemcpyHostToDevice, ctx->st));
  HC(hipMemcpyAsync(t, t_mont, E, hipMemcpyHostToDevice, ctx->st));
  if (sel_f) {
    sf = ctx->buf("gb_sf", E);
    st = ctx->buf("gb_st", E);
    HC(hipMemcpyAsync(sf, sel_f, E, hipMemcpyHostToDevice, ctx->st));
    HC(hipMemcpyAsync(st, sel_t, E, hipMemcpyHostToDevice, ctx->st));
  }
  Fr g = Fr::from_bytes(gamma_mont);
  uint32_t* dg = ctx->scal(&g, 1);
  uint32_t* flags = ctx->buf("flags", 64);
  HC(hipMemsetAsync(flags, 0, 64, ctx->st));
  const uint32_t ntiles = (uint32_t)((n + EVAL_TILE - 1) / EVAL_TILE);
  launch_builder(ctx->st, kind == KGS_GRANDPRODUCT, sel_f != nullptr, o, f, t, sf, st, dg, n,
                 ctx->buf("bt_tp", 32 * (ntiles + 1)), ctx->buf("bt_ti", 32 * (ntiles + 1)), flags);
  check_launch();
  uint32_t* hf = (uint32_t*)ctx->pin(64);
  HC(hipMemcpyAsync(out_mont, o, E, hipMemcpyDeviceToHost, ctx->st));
  HC(hipMemcpyAsync(hf, flags, 64, hipMemcpyDeviceToHost, ctx->st));
  ctx->sync();
  bool bad = hf[0] != 0;
  ctx->reset_staging();
  if (bad)
    throw KgsError(KGS_E_NOT_WELL_CALC, kind != KGS_GRANDPRODUCT ? "The grand-sum polynomial S is not well calculated"
                                                             : "The grand-product polynomial Z is not well calculated");
  API_END
}

int kgs_poly_eval(kgs_ctx_t* ctx, const uint8_t* coef_mont, uint64_t len, const uint8_t x_mont[32],
                  uint8_t out_mont[32]) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  ctx->reset_staging();
  uint32_t* a = ctx->buf("prim_a", 32 * (len ? len : 1));
  HC(hipMemcpyAsync(a, coef_mont, 32 * len, hipMemcpyHostToDevice, ctx->st));
  EvalJob j = eval_launch(*ctx, {a}, {len}, Fr::from_bytes(x_mont), 0);
  ctx->sync();
  eval_finish(j)[0].to_bytes(out_mont);
  ctx->reset_staging();
  API_END
}

int kgs_poly_div_x_sub(kgs_ctx_t* ctx, const uint8_t* coef_mont, uint64_t len, const uint8_t z_mont[32],
                       uint8_t* out_mont) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if (len < 2) throw KgsError(KGS_E_ARG, "length must be >= 2");
  ctx->reset_staging();
  uint32_t* a = ctx->buf("prim_a", 32 * len);
  uint32_t* b = ctx->buf("prim_b", 32 * len);
  uint32_t* flags = ctx->buf("flags", 64);
  HC(hipMemsetAsync(flags, 0, 64, ctx->st));
  HC(hipMemcpyAsync(a, coef_mont, 32 * len, hipMemcpyHostToDevice, ctx->st));
  const uint32_t dt = (uint32_t)((len + EVAL_TILE - 1) / EVAL_TILE);
  launch_divide(ctx->st, b, flags, a, len, xpowers(*ctx, Fr::from_bytes(z_mont)), ctx->buf("div_part", 32 * (dt + 1)),
                ctx->buf("div_carry", 32 * (dt + 1)));
  check_launch();
  uint32_t* hf = (uint32_t*)ctx->pin(64);
  HC(hipMemcpyAsync(out_mont, b, 32 * len, hipMemcpyDeviceToHost, ctx->st));
  HC(hipMemcpyAsync(hf, flags, 64, hipMemcpyDeviceToHost, ctx->st));
  ctx->sync();
  bool bad = hf[0] != 0;
  ctx->reset_staging();
  if (bad) throw KgsError(KGS_E_DOES_NOT_DIVIDE, "Polynomial does not divide");
  API_END
}

int kgs_keccak256(const uint8_t* data, uint64_t len, uint8_t out[32]) {
  host::keccak256(data, (size_t)len, out);
  return KGS_OK;
}

int kgs_bench_msm(kgs_ctx_t* ctx, const void* d_scalars_mont, uint64_t n, int reps, double* ms) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if (n > ctx->tb.npts || ctx->srs_slice_world > 1) throw KgsError(KGS_E_SRS, "MSM larger than the resident SRS (or an SRS slice)");
  uint32_t* dT = ctx->buf("msm_T", (size_t)64 * ctx->tb.c * 128);
  msm_run(ctx->st, ctx->tb, ctx->mw, (const uint32_t*)d_scalars_mont, n, dT);  // warm
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  HC(hipEventRecord(e0, ctx->st));
  for (int r = 0; r < reps; r++) msm_run(ctx->st, ctx->tb, ctx->mw, (const uint32_t*)d_scalars_mont, n, dT);
  HC(hipEventRecord(e1, ctx->st));
  HC(hipEventSynchronize(e1));
  float f = 0;
  HC(hipEventElapsedTime(&f, e0, e1));
  *ms = f;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  API_END
}

int kgs_bench_msm_phases(kgs_ctx_t* ctx, const void* d_scalars_mont, uint64_t n, int reps, double* phase_ms,
                         uint64_t* entries) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if (n > ctx->tb.npts || ctx->srs_slice_world > 1) throw KgsError(KGS_E_SRS, "MSM larger than the resident SRS (or an SRS slice)");
  uint32_t* dT = ctx->buf("msm_T", (size_t)64 * ctx->tb.c * 128);
  hipEvent_t ev[5];
  for (auto& e : ev) HC(hipEventCreate(&e));
  for (int i = 0; i < 4; i++) phase_ms[i] = 0;
  for (int r = 0; r < reps; r++) {
    msm_run(ctx->st, ctx->tb, ctx->mw, (const uint32_t*)d_scalars_mont, n, dT, ev);
    HC(hipEventSynchronize(ev[4]));
    for (int i = 0; i < 4; i++) {
      float f = 0;
      HC(hipEventElapsedTime(&f, ev[i], ev[i + 1]));
      phase_ms[i] += f;
    }
  }
  const uint32_t B = 1u << (ctx->tb.c - 1);
  uint32_t tot = 0;
  HC(hipMemcpy(&tot, ctx->mw.offsets + (B + 1), 4, hipMemcpyDeviceToHost));
  if (entries) *entries = tot;
  for (auto& e : ev) hipEventDestroy(e);
  API_END
}

int kgs_bench_ntt(kgs_ctx_t* ctx, void* d_buf, int logm, int reps, double* ms) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  CTX_LOCK(ctx);
  HC(hipSetDevice(ctx->device));
  if (logm > ctx->logM) ensure_domain(*ctx, logm);
  uint32_t* a = (uint32_t*)d_buf;
  const uint64_t m = 1ull << logm;
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  HC(hipEventRecord(e0, ctx->st));
  for (int r = 0; r < reps; r++) {
    ntt_dif(ctx->st, a, a, m, logm, nullptr, ctx->tw_fwd, ctx->logM);
    ntt_dit(ctx->st, a, a, 1, logm, ctx->tw_inv, ctx->logM, nullptr, ctx->invm + 8 * logm);
  }
  HC(hipEventRecord(e1, ctx->st));
  HC(hipEventSynchronize(e1));
  float f = 0;
  HC(hipEventElapsedTime(&f, e0, e1));
  *ms = f;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  API_END
}

}  // extern "C"
