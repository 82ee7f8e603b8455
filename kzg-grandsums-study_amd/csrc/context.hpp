// Internal interface of the prover library (not part of the C-ABI): the context, the shared
// device tables and the host-side building blocks of a proof. Shared by prover.cpp (single-GPU
// prover, C-ABI) and prover_dist.cpp (the distributed prover over a rank group).
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <algorithm>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/kgs.h"
#include "host_error.hpp"
#include "host_field.hpp"
#include "kernels.hpp"
#ifndef KGS_NO_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif

namespace kgsi {
using namespace kgs;
using host::Fq;
using host::Fr;

#define HC(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess)                                                                        \
      throw KgsError(KGS_E_HIP, std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

inline void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw KgsError(KGS_E_HIP, std::string("HIP launch error: ") + hipGetErrorString(e));
}

using host::fr_w;

// roctx ranges (rocprofv3 --marker-trace): one per prover round and per host-boundary phase, so a
// trace shows where a proof's host wall time goes next to its kernels. -DKGS_NO_ROCTX removes them.
struct Range {
  bool open = false;
  explicit Range(const char* name = nullptr) {
    if (name) push(name);
  }
  void push(const char* name) {
    pop();
#ifndef KGS_NO_ROCTX
    roctxRangePushA(name);
#endif
    open = true;
  }
  void pop() {
#ifndef KGS_NO_ROCTX
    if (open) roctxRangePop();
#endif
    open = false;
  }
  ~Range() { pop(); }
};
inline const char* const ROUND_NAMES[5] = {"kgs.round1.commit_witness", "kgs.round2.grand_poly", "kgs.round3.quotient",
                                    "kgs.round4.evaluations", "kgs.round5.openings"};

// Every device allocation goes through here (prover.cpp). KGS_DEBUG_ALLOC_LIMIT=<bytes> (fault
// injection for the tests) makes any single request above that size fail as out-of-memory.
hipError_t dev_malloc(void** p, size_t bytes);

// multisets per proof (the reference has no limit; this only bounds host-side bookkeeping)
constexpr int KGS_MAX_POLS = 1024;

#ifndef KGS_C_MAX
#define KGS_C_MAX 20
#endif

struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// Read-only device tables shared by every context on a device (one copy per device, not per
// in-flight context): the SRS window tables of a ptau (keyed by file identity and the domain they
// were loaded for) and the NTT / coset twiddle tables (the largest domain built so far serves every
// smaller one: stage tables tw[h + t] = w_2h^t do not depend on the maximum domain). Published only
// after their build has completed (stream synchronised), released when the last context drops them.
struct SrsTables {
  int device = 0;
  std::string file;  // file identity (path + size + mtime) or "mem#<id>"
  int power = -1, nbits_max = -1;
  // a rank's slice of the SRS (kgs_srs_load_ptau_slice): row 0 holds the points slice_rank +
  // slice_world * j only (slice_world == 1: the whole prefix)
  int slice_rank = 0, slice_world = 1;
  MsmTables tb;
  ~SrsTables() {
    if (tb.table) {
      hipSetDevice(device);
      hipFree(tb.table);
    }
  }
};

struct DomainTables {
  int device = 0, logM = -1;
  uint32_t* mem = nullptr;
  uint32_t *tw_fwd = nullptr, *tw_inv = nullptr, *coset_pow = nullptr, *coset_ipow = nullptr, *invm = nullptr;
  // every table of `mem` again as 9 x 29-bit limbs of x * 2^261 (10 words per element, fr29.hpp): the
  // LDS NTT passes' twiddle and scaling products (ntt_register_tw29 maps a pointer into `mem` to its
  // record here)
  uint32_t* mem29 = nullptr;
  ~DomainTables() {
    hipSetDevice(device);
    if (mem29) {
      ntt_unregister_tw29(mem);
      hipFree(mem29);
    }
    if (mem) hipFree(mem);
  }
};

extern std::mutex g_reg_mu;  // lock order: kgs_ctx::mu, then g_reg_mu
extern std::vector<std::weak_ptr<SrsTables>> g_srs_reg;
extern std::vector<std::weak_ptr<DomainTables>> g_dom_reg;

}  // namespace kgsi

using namespace kgsi;

// Rank group of the distributed prover (transports in prover_dist.cpp). wait() drains a stream that
// may hold the group's exchanges: a transport whose peers can hang (RCCL) polls it against a
// deadline instead of blocking forever.
struct kgs_group {
  int world = 1;
  virtual ~kgs_group() {}
  // blocking host all-gather: recv = world x bytes, rank-major
  virtual void allgather(int rank, const void* send, void* recv, size_t bytes) = 0;
  // device all-to-all ordered on st: chunk j of send -> rank j; chunk j of recv <- rank j
  virtual void alltoall(int rank, struct kgs_ctx& c, hipStream_t st, const void* send, void* recv, size_t chunk) = 0;
  // bytes that leave a rank in one alltoall of `chunk`-byte chunks on this transport: the chunks for
  // the W - 1 other ranks, unless the transport moves more (HostGroup without an all-to-all callback
  // all-gathers the whole send buffer)
  virtual uint64_t alltoall_wire_bytes(size_t chunk) const { return (uint64_t)chunk * (world - 1); }
  // a rank failed: unblock the others (they fail too instead of waiting forever)
  virtual void abort() {}
  // a context on `device` becomes `rank` (kgs_ctx_set_group): transports that move device data
  // between the ranks' devices directly prepare that here
  virtual void attach(int rank, int device) { (void)rank; (void)device; }
  virtual void wait(hipStream_t st) {
    const hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) throw KgsError(KGS_E_HIP, std::string("HIP error: ") + hipGetErrorString(e) + " (stream sync)");
  }
};
// seconds a rank waits for its peers in a group exchange (KGS_GROUP_TIMEOUT_S, default 120)
double group_timeout_s();

// Exchanges of the last distributed proof on a context (kgs_last_exchange): every all-to-all is
// bracketed by two events on the stream it is ordered on (its span includes waiting for the peers),
// every host all-gather by the wall clock; bytes are those leaving this rank.
struct ExchangeStats {
  int a2a_n = 0, ag_n = 0;
  double a2a_ms = 0, ag_ms = 0;
  uint64_t a2a_bytes = 0, ag_bytes = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;  // grow-only pool
  void reset() {
    a2a_n = ag_n = 0;
    a2a_ms = ag_ms = 0;
    a2a_bytes = ag_bytes = 0;
  }
  ~ExchangeStats() {
    for (auto& e : ev) {
      hipEventDestroy(e.first);
      hipEventDestroy(e.second);
    }
  }
};

struct kgs_ctx {
  // every C-ABI entry point that touches the context holds mu: a busy context blocks its caller,
  // it is never entered twice (the JS backend runs prove() calls on libuv worker threads)
  std::mutex mu;
  int device = 0;
  hipStream_t st = nullptr;
  std::map<std::string, DBuf> pool;
  // pinned staging of the host-buffer boundary: h_in receives kgs_prove's inputs (the CPU only writes
  // it, the DMA engine reads it), h_io the Montgomery write-back (the CPU reads it). KGS_STAGE_WC=1
  // makes h_in write-combined: SDMA reads that at ~55 GB/s against ~30 GB/s from coherent pinned
  // memory alone (profiles/r05/d2h_engine.txt), but the host copy into it is slower and a proof
  // measured the same either way (profiles/r05/stage_wc_ab.txt), so it is off by default
  uint8_t* h_in = nullptr;
  size_t h_in_bytes = 0;
  uint8_t* h_io = nullptr;
  size_t h_io_bytes = 0;
  // pinned staging
  uint8_t* h_pin = nullptr;
  size_t h_pin_bytes = 0;
  size_t h_pin_off = 0;
  uint32_t* d_scal = nullptr;  // device scalar area
  size_t d_scal_off = 0;
  static constexpr size_t SCAL_BYTES = 1 << 16;
  // SRS (shared, read-only) and this context's views of it
  std::shared_ptr<SrsTables> srs;
  int srs_power = -1;
  int nbits_max = -1;
  MsmTables tb;
  MsmWork mw;
  uint64_t work_npts = 0;  // MSM work buffers (both lanes) are sized for this many points
  int msm_slots = 0;       // commitments in flight per proof (msm_T slots)
  // second MSM lane: independent commitments of one round (R1's F_i/T_i, R5's two W) alternate
  // between st and st2 (own work buffers), so one MSM's latency-bound tail overlaps the other's
  // bucket accumulation
  hipStream_t st2 = nullptr;
  hipStream_t st_copy = nullptr;  // kgs_prove's input DMAs (vectors 1..)
  // the Montgomery write-back (prover.js:147-148): its own stream, so that it never sits between
  // the input DMAs on st_copy; each vector's D2H waits only for that vector's conversion
  hipStream_t st_wb = nullptr;
  std::vector<hipEvent_t> ev_wb;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  std::vector<hipEvent_t> ev_in;  // kgs_prove: one per input vector DMA'd on the copy stream
  MsmWork mw2;
  int msm_lanes = 2;  // kgs_ctx_set_msm_lanes
  bool ref_quirks = true;  // kgs_ctx_set_reference_quirks (ref_quirks.cpp); default on
  uint64_t msm_nseg_max = 0;
  // domain tables (M = 2^logM; shared) and this context's views of them
  std::shared_ptr<DomainTables> dom;
  int logM = -1;
  uint32_t *tw_fwd = nullptr, *tw_inv = nullptr, *coset_pow = nullptr, *coset_ipow = nullptr, *invm = nullptr;
  std::map<std::pair<int, int>, uint32_t*> nxm1;  // (nbits, lcs) -> 1/(n(x-1)) on the coset (bitrev)
  std::vector<double> timing;
  // MSM point-range sharding (kgs_ctx_set_shard): world > 1 splits every commitment MSM
  int shard_rank = 0, shard_world = 1;
  kgs_allgather_fn shard_fn = nullptr;
  void* shard_user = nullptr;
  // distributed prover (kgs_ctx_set_group): every vector sharded over the group's ranks
  kgs_group* group = nullptr;
  int group_rank = 0;
  int srs_slice_rank = 0, srs_slice_world = 1;  // of the loaded SRS (SrsTables::slice_*)
  std::map<std::string, uint32_t*> dist_tabs;  // per-rank coset / 1/(n(x-1)) tables (pool buffers)
  ExchangeStats xs;                             // exchanges of the last distributed proof
  bool dist_err_agreed = false;  // the distributed proof's current failure is the same on every rank

  ~kgs_ctx() {
    hipSetDevice(device);
    // every stream may still read pool buffers or pinned staging: drain all before freeing. A drain
    // that fails is reported here, naming the stream: HIP errors are sticky, and unreported the fault
    // would surface at the next checked call of whatever runs next in the process (round 5's fault
    // surfaced that way in the NEXT test's first copy, profiles/r05/boundary/feed_per_piece_dma_fault.log)
    const char* names[4] = {"main", "lane 2", "input copy", "write-back"};
    const hipStream_t ss[4] = {st, st2, st_copy, st_wb};
    for (int i = 0; i < 4; i++) {
      if (!ss[i]) continue;
      const hipError_t e = hipStreamSynchronize(ss[i]);
      if (e != hipSuccess)
        fprintf(stderr, "kgs: context on device %d: its %s stream failed while draining at destruction: %s\n", device,
                names[i], hipGetErrorString(e));
    }
    for (auto& kv : pool) hipFree(kv.second.p);
    if (h_pin) hipHostFree(h_pin);
    if (h_io) hipHostFree(h_io);
    if (h_in) hipHostFree(h_in);
    if (ev_fork) hipEventDestroy(ev_fork);
    if (ev_join) hipEventDestroy(ev_join);
    for (hipEvent_t e : ev_in) hipEventDestroy(e);
    for (hipEvent_t e : ev_wb) hipEventDestroy(e);
    if (st_wb) hipStreamDestroy(st_wb);
    if (st_copy) hipStreamDestroy(st_copy);
    if (st2) hipStreamDestroy(st2);
    if (st) hipStreamDestroy(st);
    {
      std::lock_guard<std::mutex> lk(g_reg_mu);  // shared tables are released under the registry lock
      srs.reset();
      dom.reset();
    }
  }

  // A failed (re)allocation leaves the slot empty (bytes = 0), never a stale size over a freed block.
  uint32_t* buf(const std::string& name, size_t bytes) {
    DBuf& b = pool[name];
    if (b.bytes < bytes) {
      if (b.p) {
        sync();  // any stream may still use the old block
        HC(hipFree(b.p));
        b.p = nullptr;
        b.bytes = 0;
      }
      const size_t sz = bytes < 64 ? 64 : bytes;
      HC(dev_malloc(&b.p, sz));
      b.bytes = sz;
    }
    return (uint32_t*)b.p;
  }
  uint8_t* io_in(size_t bytes) {
    if (h_in_bytes < bytes) {
      if (h_in) {
        sync();
        HC(hipHostFree(h_in));
        h_in = nullptr;
        h_in_bytes = 0;
      }
      static const bool wc = [] {
        const char* e = getenv("KGS_STAGE_WC");
        return e && !strcmp(e, "1");
      }();
      HC(hipHostMalloc((void**)&h_in, bytes, wc ? hipHostMallocWriteCombined : hipHostMallocDefault));
      h_in_bytes = bytes;
    }
    return h_in;
  }
  uint8_t* io(size_t bytes) {
    if (h_io_bytes < bytes) {
      if (h_io) {
        sync();
        HC(hipHostFree(h_io));
        h_io = nullptr;
        h_io_bytes = 0;
      }
      HC(hipHostMalloc((void**)&h_io, bytes, hipHostMallocDefault));
      h_io_bytes = bytes;
    }
    return h_io;
  }
  void ensure_pin(size_t bytes) {
    if (h_pin_bytes >= bytes) return;
    if (h_pin) {
      sync();
      HC(hipHostFree(h_pin));
      h_pin = nullptr;
      h_pin_bytes = 0;
      h_pin_off = 0;
    }
    HC(hipHostMalloc((void**)&h_pin, bytes, hipHostMallocDefault));
    h_pin_bytes = bytes;
  }
  // bump-allocated pinned region (valid until reset_staging(), i.e. until the next sync point)
  uint8_t* pin(size_t bytes) {
    bytes = (bytes + 63) & ~size_t(63);
    if (h_pin_off + bytes > h_pin_bytes) throw KgsError(KGS_E_ARG, "pinned staging exhausted");
    uint8_t* p = h_pin + h_pin_off;
    h_pin_off += bytes;
    return p;
  }
  // copy host scalars to the device scalar area; returns the device pointer
  uint32_t* scal(const Fr* v, int count) {
    size_t bytes = 32 * (size_t)count;
    if (d_scal_off + bytes > SCAL_BYTES) throw KgsError(KGS_E_ARG, "scalar staging exhausted");
    uint8_t* h = pin(bytes);
    for (int i = 0; i < count; i++) v[i].to_bytes(h + 32 * i);
    uint32_t* d = d_scal + d_scal_off / 4;
    d_scal_off += bytes;
    HC(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
    return d;
  }
  void sync() {
    if (group) group->wait(st);  // the main stream carries the group's exchanges
    else HC(hipStreamSynchronize(st));
    if (st2) HC(hipStreamSynchronize(st2));
    if (st_copy) HC(hipStreamSynchronize(st_copy));
    if (st_wb) HC(hipStreamSynchronize(st_wb));
  }
  void reset_staging() {
    sync();
    h_pin_off = 0;
    d_scal_off = 0;
  }
  void use_srs(const std::shared_ptr<SrsTables>& s) {
    srs = s;
    tb = s ? s->tb : MsmTables{};
    srs_power = s ? s->power : -1;
    nbits_max = s ? s->nbits_max : -1;
    srs_slice_rank = s ? s->slice_rank : 0;
    srs_slice_world = s ? s->slice_world : 1;
  }
  void use_domain(const std::shared_ptr<DomainTables>& d) {
    dom = d;
    logM = d->logM;
    tw_fwd = d->tw_fwd;
    tw_inv = d->tw_inv;
    coset_pow = d->coset_pow;
    coset_ipow = d->coset_ipow;
    invm = d->invm;
  }
};


namespace kgsi {

// ------------------------------------------------------------------ building blocks (prover.cpp)
// twin: also the tables' 29-bit twin (false only for the reference-quirks replay's growth)
void ensure_domain(kgs_ctx& c, int logM, bool twin = true);
void ensure_twin(kgs_ctx& c);  // the context's domain gets its twin if it was grown without one
uint32_t* get_nxm1(kgs_ctx& c, int nbits, int lcs);
void intt_nat(kgs_ctx& c, uint32_t* out, const uint32_t* in, int logm, hipStream_t st = nullptr);
// coefficients (len <= 2^lcs) -> coset evaluations p(g w^i), bit-reversed order
void coset_fwd(kgs_ctx& c, uint32_t* out, const uint32_t* in, uint64_t len, int lcs, hipStream_t st = nullptr);
// bit-reversed coset evaluations ALREADY SCALED BY 1/2^lcs -> natural coefficients (in place allowed);
// the quotient takes its 1/cs from the Z_H scalars and get_nxm1's table
void coset_inv_prescaled(kgs_ctx& c, uint32_t* out, const uint32_t* in, int lcs);

// reference-quirks mode (ref_quirks.cpp; kgs_ctx_set_reference_quirks)
uint32_t* ref_quirks_probe(kgs_ctx& c, uint64_t n, const std::vector<const uint32_t*>& ops, const uint32_t* Q,
                           uint64_t qlen);
bool ref_quirks_needed(const uint32_t* probe, size_t nops, uint64_t n);
bool ref_quotient_is_zero(const uint32_t* probe);
uint32_t* ref_quirks_quotient(kgs_ctx& c, bool gs, bool sel, bool lookup, int nbits, const Fr& alpha, const Fr& gamma,
                              const uint32_t* dF, const uint32_t* dT, const uint32_t* dS, const uint32_t* dSF,
                              const uint32_t* dST, uint64_t& qlen, uint32_t*& fmut);

// MSM commitment: device Pippenger -> c bit-sum points T_k (this rank's partial, pinned host)
struct Commit {
  uint8_t* h_T = nullptr;   // pinned, c x 128 B (this rank's partial)
  uint64_t N = 0;
  uint8_t* h_T2 = nullptr;  // second point range's partial (commit_launch_split), or nullptr
};
void shard_range(uint64_t n, int rank, int world, uint64_t& lo, uint64_t& hi);
void fork_lanes(kgs_ctx& c);
Commit commit_launch(kgs_ctx& c, const uint32_t* scalars, uint64_t N, int slot, int lane = 0);
// latency mode (two MSM lanes, one unsharded context): points [0, cut) on lane 0 and [cut, N) on
// lane 1 (slots slot, slot + 1); the two partials are summed by commits_finish. Otherwise the same
// as commit_launch on `lane`.
Commit commit_launch_split(kgs_ctx& c, const uint32_t* scalars, uint64_t N, uint64_t cut, int slot);
bool split_commits(const kgs_ctx& c);
// MSM over `count` scalars whose SRS points are pbase + pstride * i (a rank's slice of a
// distributed polynomial); N = the polynomial's global point count (0: infinity)
Commit commit_launch_slice(kgs_ctx& c, const uint32_t* scalars, uint64_t count, uint64_t pbase, uint64_t pstride,
                           uint64_t N, int slot, int lane = 0);
void combine_partials(const uint8_t* T_all, size_t part_stride, int nparts, int cc, uint8_t out[64]);
// all-gather of per-rank partials (nullptr: this rank alone) -> affine LEM commitments
using HostAllgather = std::function<void(const void* send, void* recv, size_t bytes)>;
void commits_finish(kgs_ctx& c, const std::vector<Commit>& cms, std::vector<uint8_t*> outs);
void commits_finish_with(kgs_ctx& c, const std::vector<Commit>& cms, std::vector<uint8_t*> outs, int world,
                         const HostAllgather& ag);
void commit_finish(kgs_ctx& c, const Commit& cm, uint8_t out[64]);

// Horner evaluations (tile partials on the device, tile combine on the host)
struct EvalJob {
  std::vector<const uint32_t*> src;
  std::vector<uint64_t> len;
  uint8_t* h_part = nullptr;
  uint32_t ntiles = 0;
  Fr x;
};
uint32_t* xpowers(kgs_ctx& c, const Fr& x);
void fr29_record(const Fr& x, Fr out[2]);
EvalJob eval_launch(kgs_ctx& c, const std::vector<const uint32_t*>& src, const std::vector<uint64_t>& len, const Fr& x,
                    int slot);
std::vector<Fr> eval_finish(const EvalJob& j);

// out[i] = sum_k coef_k * src_k[i] (zero beyond len_k) + (i == 0 ? c0 : 0), any number of terms
struct LcTerms {
  std::vector<const uint32_t*> src;
  std::vector<uint64_t> len;
  std::vector<Fr> coef;
  Fr c0 = Fr::zero();
  void add(const uint32_t* s, uint64_t l, const Fr& k) {
    src.push_back(s);
    len.push_back(l);
    coef.push_back(k);
  }
};
void run_lincomb(hipStream_t st, uint32_t* out, uint64_t n, const LcTerms& t);

struct ProveIn {
  int kind, nbits, npols;
  std::vector<const uint32_t*> f_std, t_std;  // device, standard form
  const uint32_t *sel_f = nullptr, *sel_t = nullptr;  // device, Montgomery (nullptr: unselected)
  std::vector<uint8_t*> mont_f_out, mont_t_out;  // host outputs (may be empty)
  std::function<void()> after_round1;             // called once round 1 is synchronised (write-back on st_wb)
  // kgs_prove: per input vector (F_i at 2i, T_i at 2i + 1, then selF, selT) an event the main stream
  // waits for before the vector's first kernel, or nullptr (already ordered on the main stream)
  std::vector<hipEvent_t> ready;
  // kgs_prove: blocks until vector v's DMA (and ready[v]) has been enqueued; null: all already are
  std::function<void(size_t)> input_issued;
};
enum R5Poly { R5_S, R5_Q, R5_F, R5_T, R5_SELF, R5_SELT, R5_POLT };
struct R5Term {
  R5Poly id;
  int idx;  // vector index for R5_F / R5_T
  Fr coef;
};
struct R5 {
  Fr c0;
  std::vector<R5Term> terms;
};
R5 round5_terms(bool gs, bool sel, int k, int nbits, const Fr& alpha, const Fr& beta, const Fr& gamma, const Fr& v,
                const Fr& xi, const std::vector<Fr>& fx, const std::vector<Fr>& tx, const Fr& sFx, const Fr& sTx,
                const Fr& sxiw, bool lookup, const Fr* fxi_override = nullptr);

void prove_impl(kgs_ctx& c, const ProveIn& in, uint8_t* com_out, uint8_t* ev_out);
// the distributed prover (prover_dist.cpp): same inputs and outputs as prove_impl on every rank
void prove_dist_impl(kgs_ctx& c, const ProveIn& in, uint8_t* com_out, uint8_t* ev_out);
void prove_dist_group(kgs_ctx& c, const ProveIn& in, uint8_t* com_out, uint8_t* ev_out);

// host copies between pageable caller buffers and pinned staging, split over threads
struct CopyJob {
  uint8_t* dst;
  const uint8_t* src;
  size_t len;
};
void par_copy(const std::vector<CopyJob>& jobs);
// one vector into pinned staging; ready(offset, len) on the calling thread per `dma`-byte span, in
// order, once that span is copied (prover.cpp)
void stream_copy(uint8_t* dst, const uint8_t* src, size_t len, size_t dma, const std::function<void(size_t, size_t)>& ready);

}  // namespace kgsi
