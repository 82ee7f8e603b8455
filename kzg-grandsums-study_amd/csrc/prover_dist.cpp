// The distributed prover: one proof over a group of W ranks (one context per rank, one GPU each
// on a node), every vector sharded, so that the NTTs, the builder, the quotient, the Horner
// evaluations, the synthetic divisions AND the MSMs all shrink as 1/W per rank (SURVEY.md §8e;
// north_star: "the MSM and NTT shard ... by scalar/point range and by butterfly stage").
//
// Layouts and the exchange steps are specified (and checked on CPU) by tests/test_dist_layouts.py;
// dist.hip holds the rank-local kernels. Per grand-sum proof (k = 1, no selectors) the data
// exchanges are 10 all-to-alls of one vector each (RCCL send/recv over xGMI, stream-ordered) plus a
// handful of small host all-gathers (rank totals, halos, Horner partials, division carries, MSM
// bit-sum partials). Every rank ends with the identical proof; inputs are the full vectors on every
// rank (each rank reads only its slices), outputs identical to the single-GPU prover byte for byte.
//
//   round 1  F_i, T_i: H-evaluations gathered in E layout -> iDFT (E -> CYCLIC) -> MSM over the
//            rank's CYCLIC slice (SRS points r, r + W, ...)
//   round 2  builder on BLOCK slices + one all-gather of rank totals (prefix offsets, the "not well
//            calculated" check) -> BLOCK -> E -> iDFT -> S (CYCLIC); coset DFTs CYCLIC -> E
//   round 3  divisibility check on BLOCK (one halo element), quotient on E (rot halo elements per
//            block), inverse coset DFT E -> CYCLIC -> MSM
//   round 4  Horner on CYCLIC slices at x^W, combined as sum_r x^r v_r after one all-gather
//   round 5  linear combination on CYCLIC -> BLOCK -> synthetic division with one all-gather of
//            carries (Polynomial.divByXSubValue, polynomial.js:814-851) -> MSM over BLOCK ranges
//
// Transports (kgs_group): RCCL (one process per GPU, production), in-process (several contexts of
// one process: tests on one GPU, or one process driving several GPUs), host callback (any
// all-gather, e.g. torch.distributed gloo; device data staged through the host).
#include <condition_variable>
#include <thread>
#include <rccl/rccl.h>

#include "context.hpp"
#include "transcript.hpp"

using namespace kgs;
using namespace kgsi;

// ------------------------------------------------------------------ rank groups
// (the kgs_group interface is in context.hpp: kgs_ctx::sync drains the main stream through it)
double group_timeout_s() {
  static const double t = [] {
    const char* e = getenv("KGS_GROUP_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0 ? v : 120.0;
  }();
  return t;
}

namespace {

// several contexts of one process, driven by one host thread per rank
struct LocalGroup : kgs_group {
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<const void*> sp;
  std::vector<int> dev;
  std::vector<int> attached;  // device of each attached rank (-1: none yet)

  explicit LocalGroup(int w) : sp(w), dev(w), attached(w, -1) { world = w; }

  // `a` reads from / writes to `b`'s memory in the all-to-all (hipMemcpyPeerAsync): without peer
  // access the runtime would stage the copy through the host, so a pair without it fails up front
  static void enable_peer(int a, int b) {
    int can = 0;
    HC(hipDeviceCanAccessPeer(&can, a, b));
    if (!can)
      throw KgsError(KGS_E_COMM, "in-process rank group: device " + std::to_string(a) + " has no peer access to device " +
                                     std::to_string(b) + " (hipDeviceCanAccessPeer); use one process per GPU (RCCL)");
    int cur = 0;
    HC(hipGetDevice(&cur));
    HC(hipSetDevice(a));
    const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
    (void)hipGetLastError();
    HC(hipSetDevice(cur));
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
      throw KgsError(KGS_E_COMM, std::string("in-process rank group: hipDeviceEnablePeerAccess failed: ") + hipGetErrorString(e));
  }
  void attach(int rank, int device) override {
    std::lock_guard<std::mutex> lk(mu);
    for (int j = 0; j < world; j++)
      if (j != rank && attached[j] >= 0 && attached[j] != device) {
        enable_peer(device, attached[j]);
        enable_peer(attached[j], device);
      }
    attached[rank] = device;
  }

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) throw KgsError(KGS_E_COMM, "rank group aborted");
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return;
    }
    if (!cv.wait_for(lk, std::chrono::duration<double>(group_timeout_s()), [&] { return gen != g || broken; })) {
      broken = true;
      cv.notify_all();
      throw KgsError(KGS_E_COMM, "rank group barrier timed out");
    }
    if (broken) throw KgsError(KGS_E_COMM, "rank group aborted");
  }
  void abort() override {
    std::lock_guard<std::mutex> lk(mu);
    broken = true;
    cv.notify_all();
  }
  void allgather(int rank, const void* send, void* recv, size_t bytes) override {
    sp[rank] = send;
    barrier();
    for (int j = 0; j < world; j++) memcpy((uint8_t*)recv + (size_t)j * bytes, sp[j], bytes);
    barrier();  // the senders' buffers stay valid until every rank has copied
  }
  void alltoall(int rank, kgs_ctx& c, hipStream_t st, const void* send, void* recv, size_t chunk) override {
    HC(hipStreamSynchronize(st));  // send is complete
    sp[rank] = send;
    dev[rank] = c.device;
    barrier();
    for (int j = 0; j < world; j++) {
      uint8_t* dst = (uint8_t*)recv + (size_t)j * chunk;
      const uint8_t* src = (const uint8_t*)sp[j] + (size_t)rank * chunk;
      if (dev[j] == c.device) HC(hipMemcpyAsync(dst, src, chunk, hipMemcpyDeviceToDevice, st));
      else HC(hipMemcpyPeerAsync(dst, c.device, src, dev[j], chunk, st));  // peer access: attach()
    }
    HC(hipStreamSynchronize(st));
    barrier();  // nobody overwrites a send buffer a peer is still reading
  }
};

// host callbacks (torch.distributed gloo, MPI ...): device data staged through the host. With an
// all-to-all callback each rank sends chunk j to rank j and receives one chunk from each rank
// ((W - 1) / W of its vector leaves it); with only the all-gather, every rank receives every rank's
// whole vector (W x the data) and keeps its chunks.
struct HostGroup : kgs_group {
  kgs_allgather_fn fn;
  kgs_alltoall_fn a2a_fn;
  void* user;
  std::vector<uint8_t> h_send, h_recv;
  HostGroup(int w, kgs_allgather_fn f, kgs_alltoall_fn a, void* u) : fn(f), a2a_fn(a), user(u) { world = w; }
  void allgather(int, const void* send, void* recv, size_t bytes) override {
    if (fn(user, (const uint8_t*)send, (uint8_t*)recv, bytes) != 0) throw KgsError(KGS_E_COMM, "group all-gather failed");
  }
  uint64_t alltoall_wire_bytes(size_t chunk) const override {
    return a2a_fn ? (uint64_t)chunk * (world - 1) : (uint64_t)chunk * world * (world - 1);
  }
  void alltoall(int rank, kgs_ctx&, hipStream_t st, const void* send, void* recv, size_t chunk) override {
    const size_t bytes = chunk * world;
    if (h_send.size() < bytes) h_send.resize(bytes);
    HC(hipMemcpyAsync(h_send.data(), send, bytes, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    if (a2a_fn) {
      if (h_recv.size() < bytes) h_recv.resize(bytes);
      if (a2a_fn(user, h_send.data(), h_recv.data(), (uint64_t)chunk) != 0) throw KgsError(KGS_E_COMM, "group all-to-all failed");
      HC(hipMemcpyAsync(recv, h_recv.data(), bytes, hipMemcpyHostToDevice, st));
    } else {
      if (h_recv.size() < bytes * world) h_recv.resize(bytes * world);
      allgather(rank, h_send.data(), h_recv.data(), bytes);
      for (int j = 0; j < world; j++)
        HC(hipMemcpyAsync((uint8_t*)recv + (size_t)j * chunk, h_recv.data() + (size_t)j * bytes + (size_t)rank * chunk,
                          chunk, hipMemcpyHostToDevice, st));
    }
    HC(hipStreamSynchronize(st));
  }
};

#define NC(x)                                                                                           \
  do {                                                                                                  \
    ncclResult_t r_ = (x);                                                                              \
    if (r_ != ncclSuccess) throw KgsError(KGS_E_COMM, std::string("RCCL error: ") + ncclGetErrorString(r_) + " at " #x); \
  } while (0)

// one process per GPU: RCCL communicator, all-to-all as grouped send/recv on the prover's stream
struct RcclGroup : kgs_group {
  ncclComm_t comm = nullptr;
  int device = 0;
  hipStream_t st_small = nullptr;
  void* d_small = nullptr;
  size_t small_bytes = 0;
  ~RcclGroup() override {
    hipSetDevice(device);
    if (comm) ncclCommDestroy(comm);
    if (d_small) hipFree(d_small);
    if (st_small) hipStreamDestroy(st_small);
  }
  void allgather(int rank, const void* send, void* recv, size_t bytes) override {
    HC(hipSetDevice(device));
    if (!comm) throw KgsError(KGS_E_COMM, "rank group aborted");
    if (small_bytes < bytes * (world + 1)) {
      if (d_small) HC(hipFree(d_small));
      d_small = nullptr;
      small_bytes = 0;
      HC(dev_malloc(&d_small, bytes * (world + 1)));
      small_bytes = bytes * (world + 1);
    }
    uint8_t* ds = (uint8_t*)d_small;
    HC(hipMemcpyAsync(ds, send, bytes, hipMemcpyHostToDevice, st_small));
    NC(ncclAllGather(ds, ds + bytes, bytes, ncclUint8, comm, st_small));
    HC(hipMemcpyAsync(recv, ds + bytes, bytes * world, hipMemcpyDeviceToHost, st_small));
    wait(st_small);
    (void)rank;
  }
  // RCCL collectives are stream-ordered: a peer that never joins leaves the stream pending forever
  // (and ncclCommAbort on the failing rank does not release the others). Poll the stream and the
  // communicator's asynchronous error against the group deadline; on expiry or error abort this
  // rank's communicator too and fail, so every rank of a broken group ends with an error.
  void wait(hipStream_t st) override {
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(group_timeout_s());
    for (unsigned spin = 0;; spin++) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) throw KgsError(KGS_E_HIP, std::string("HIP error: ") + hipGetErrorString(q) + " (stream query)");
      ncclResult_t ae = ncclSuccess;
      if (comm && ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
        abort();
        throw KgsError(KGS_E_COMM, std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae));
      }
      if (!comm) throw KgsError(KGS_E_COMM, "rank group aborted");
      if (std::chrono::steady_clock::now() > t_end) {
        abort();
        throw KgsError(KGS_E_COMM, "rank group exchange timed out (a peer rank failed or hung; KGS_GROUP_TIMEOUT_S)");
      }
      if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  void alltoall(int, kgs_ctx&, hipStream_t st, const void* send, void* recv, size_t chunk) override {
    if (!comm) throw KgsError(KGS_E_COMM, "rank group aborted");
    NC(ncclGroupStart());
    for (int j = 0; j < world; j++) {
      NC(ncclSend((const uint8_t*)send + (size_t)j * chunk, chunk, ncclUint8, j, comm, st));
      NC(ncclRecv((uint8_t*)recv + (size_t)j * chunk, chunk, ncclUint8, j, comm, st));
    }
    NC(ncclGroupEnd());
  }
  void abort() override {
    if (comm) ncclCommAbort(comm);
    comm = nullptr;
  }
};

int ilog2(uint64_t x) {
  int l = 0;
  while ((1ull << l) < x) l++;
  return l;
}

}  // namespace

// ------------------------------------------------------------------ the distributed prover
namespace kgsi {



namespace {

struct Dist {
  kgs_ctx& c;
  kgs_group& g;
  const int W, r, logW;
  Dist(kgs_ctx& cc) : c(cc), g(*cc.group), W(cc.group->world), r(cc.group_rank), logW(ilog2(cc.group->world)) {}

  // every exchange is counted in c.xs (kgs_last_exchange): all-to-alls by two events on the stream,
  // host all-gathers by the wall clock; bytes leaving this rank
  void a2a(const uint32_t* send, uint32_t* recv, uint64_t chunk_elems) {
    ExchangeStats& x = c.xs;
    if ((int)x.ev.size() <= x.a2a_n) {
      hipEvent_t e0, e1;
      HC(hipEventCreate(&e0));
      HC(hipEventCreate(&e1));
      x.ev.push_back({e0, e1});
    }
    const auto& ev = x.ev[x.a2a_n++];
    HC(hipEventRecord(ev.first, c.st));
    g.alltoall(r, c, c.st, send, recv, (size_t)32 * chunk_elems);
    HC(hipEventRecord(ev.second, c.st));
    x.a2a_bytes += g.alltoall_wire_bytes((size_t)32 * chunk_elems);  // what the transport moved
  }
  void allgather(const void* s, void* rv, size_t b) {
    const auto t0 = std::chrono::steady_clock::now();
    g.allgather(r, s, rv, b);
    c.xs.ag_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c.xs.ag_n++;
    c.xs.ag_bytes += (uint64_t)b * (W - 1);
  }
  // after the proof's last sync: the all-to-all spans from their events
  void finish_stats() {
    ExchangeStats& x = c.xs;
    x.a2a_ms = 0;
    for (int i = 0; i < x.a2a_n; i++) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, x.ev[i].first, x.ev[i].second) == hipSuccess) x.a2a_ms += ms;
      else (void)hipGetLastError();
    }
  }
  // per-rank coset tables g^(+-(r + W i)), i < Ml, cached by (sign, logMl)
  uint32_t* coset_tab(int logMl, bool inverse) {
    const std::string key = std::string(inverse ? "d_cinv_" : "d_cfwd_") + std::to_string(logMl) + "_" +
                            std::to_string(W) + "_" + std::to_string(r);
    auto it = c.dist_tabs.find(key);
    if (it != c.dist_tabs.end()) return it->second;
    const uint64_t Ml = 1ull << logMl;
    uint32_t* t = c.buf(key, 32 * Ml);
    Fr g5 = Fr::from_u64(5);
    if (inverse) g5 = g5.inverse();
    Fr k[2] = {g5.pow_u64((uint64_t)W), g5.pow_u64((uint64_t)r)};
    uint32_t* d = c.scal(k, 2);
    launch_powers(c.st, t, Ml, d, d + 8);
    check_launch();
    c.dist_tabs[key] = t;
    return t;
  }
  // E (natural inside blocks) -> CYCLIC, scaled by 1/N and, for a coset, by g^-(global index)
  void inv_e_to_cyc(uint32_t* out, const uint32_t* inE, int logN, bool coset) {
    const int logMl = logN - logW;
    const uint64_t Ml = 1ull << logMl;
    uint32_t* send = c.buf("d_send", 32 * Ml);
    uint32_t* recv = c.buf("d_recv", 32 * Ml);
    launch_dinv_wdft_pack(c.st, send, inE, logMl, W, r, c.tw_inv, logN);
    check_launch();
    a2a(send, recv, Ml / W);
    ntt_dit(c.st, out, recv, 0, logMl, c.tw_inv, c.logM, coset ? coset_tab(logMl, true) : nullptr, c.invm + 8 * logN);
    check_launch();
  }
  // CYCLIC (in_len local coefficients, zero beyond) -> E evaluations (coset: g^(global index) first)
  void fwd_cyc_to_e(uint32_t* outE, const uint32_t* inC, uint64_t in_len, int logN, bool coset) {
    const int logMl = logN - logW;
    const uint64_t Ml = 1ull << logMl;
    uint32_t* Z = c.buf("d_Z", 32 * Ml);
    uint32_t* send = c.buf("d_send", 32 * Ml);
    uint32_t* recv = c.buf("d_recv", 32 * Ml);
    ntt_dif(c.st, Z, inC, in_len, logMl, coset ? coset_tab(logMl, false) : nullptr, c.tw_fwd, c.logM);
    launch_dfwd_pack(c.st, send, Z, logMl, W, r, c.tw_fwd, logN);
    check_launch();
    a2a(send, recv, Ml / W);
    launch_dfwd_wdft(c.st, outE, recv, logMl, W, c.tw_fwd, logN);
    check_launch();
  }
  void block_to_e(uint32_t* outE, const uint32_t* inB, uint64_t Ml) { a2a(inB, outE, Ml / W); }
  // BLOCK -> CYCLIC (the inverse of cyc_to_block): send chunk d = the block's indices = d mod W; the
  // received chunks, in source-rank order, are the cyclic slice in natural order
  void block_to_cyc(uint32_t* outC, const uint32_t* inB, uint64_t Lb) {
    uint32_t* send = c.buf("d_send", 32 * Lb);
    launch_pack_b2c(c.st, send, inB, Lb, W);
    check_launch();
    a2a(send, outC, Lb / W);
  }
  void cyc_to_block(uint32_t* outB, const uint32_t* inC, uint64_t Lb) {
    uint32_t* recv = c.buf("d_recv", 32 * Lb);
    a2a(inC, recv, Lb / W);
    launch_unpack_c2b(c.st, outB, recv, Lb, W);
    check_launch();
  }
  std::vector<Fr> gather_fr(const std::vector<Fr>& mine) {
    std::vector<uint8_t> s(32 * mine.size()), all(32 * mine.size() * W);
    for (size_t i = 0; i < mine.size(); i++) mine[i].to_bytes(s.data() + 32 * i);
    allgather(s.data(), all.data(), s.size());
    std::vector<Fr> out(mine.size() * W);
    for (size_t i = 0; i < out.size(); i++) out[i] = Fr::from_bytes(all.data() + 32 * i);
    return out;  // rank-major
  }
  uint32_t gather_or(uint32_t mine) {
    std::vector<uint32_t> all(W);
    allgather(&mine, all.data(), 4);
    uint32_t o = 0;
    for (uint32_t v : all) o |= v;
    return o;
  }
  HostAllgather host_ag() {
    return [this](const void* s, void* rv, size_t b) { allgather(s, rv, b); };
  }
  // Polynomial.degree (polynomial.js:212-226) of CYCLIC-sliced polynomials (rank r holds coefficients
  // r + W j, j < Ml): the highest nonzero global index over all ranks, 0 for the zero polynomial
  std::vector<uint64_t> degrees_cyc(const std::vector<const uint32_t*>& ops, uint64_t Ml) {
    const size_t m = ops.size();
    uint32_t* d = c.buf("d_qdeg", 4 * 16);
    HC(hipMemsetAsync(d, 0, 4 * 16, c.st));
    for (size_t i = 0; i < m; i++) launch_degree(c.st, d + i, ops[i], Ml);
    check_launch();
    uint8_t* h = c.pin(64 + 32 * m);
    HC(hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, c.st));
    for (size_t i = 0; i < m; i++) HC(hipMemcpyAsync(h + 64 + 32 * i, ops[i], 32, hipMemcpyDeviceToHost, c.st));
    HC(hipStreamSynchronize(c.st));
    std::vector<int64_t> mine(m);
    for (size_t i = 0; i < m; i++) {
      const uint32_t j = ((const uint32_t*)h)[i];
      bool nz0 = false;
      for (int b = 0; b < 32; b++) nz0 |= h[64 + 32 * i + b] != 0;
      mine[i] = j ? (int64_t)r + (int64_t)W * j : (nz0 ? (int64_t)r : -1);
    }
    std::vector<int64_t> all(m * W);
    allgather(mine.data(), all.data(), 8 * m);
    std::vector<uint64_t> deg(m, 0);
    for (size_t i = 0; i < m; i++)
      for (int q = 0; q < W; q++) deg[i] = std::max<int64_t>((int64_t)deg[i], all[q * m + i]);
    return deg;
  }
  // the full natural-order length-W*Ml vector of a CYCLIC-sliced polynomial, on this rank's device
  // (reference-quirks replay only: a host all-gather of the slices)
  uint32_t* gather_cyc(const uint32_t* sliceC, uint64_t Ml, const std::string& name) {
    std::vector<uint8_t> mine((size_t)32 * Ml), all((size_t)32 * Ml * W), full((size_t)32 * Ml * W);
    HC(hipMemcpyAsync(mine.data(), sliceC, mine.size(), hipMemcpyDeviceToHost, c.st));
    HC(hipStreamSynchronize(c.st));
    allgather(mine.data(), all.data(), mine.size());
    for (int q = 0; q < W; q++)
      for (uint64_t j = 0; j < Ml; j++)
        memcpy(&full[(size_t)32 * (q + W * j)], &all[(size_t)32 * (q * Ml + j)], 32);
    uint32_t* out = c.buf(name, full.size());
    HC(hipMemcpyAsync(out, full.data(), full.size(), hipMemcpyHostToDevice, c.st));
    HC(hipStreamSynchronize(c.st));
    return out;
  }
};

}  // namespace

// Rank-local preconditions (SRS loaded and large enough, the loaded SRS slice matching this rank,
// pinned staging): a rank failing one of them must not leave its peers waiting in the first
// exchange, so every rank decides them together — one all-gather of each rank's first failure, and
// every rank throws the lowest failing rank's error (the group stays usable: nothing was exchanged).
void dist_preconditions(kgs_ctx& c, const ProveIn& in) {
  const int W = c.group->world, r = c.group_rank;
  struct Verdict {
    int32_t code;
    char msg[252];
  } mine{};
  try {
    const int nbits = in.nbits, k = in.npols;
    const int logW = ilog2(W);
    if ((1 << logW) != W || W > 16) throw KgsError(KGS_E_ARG, "distributed prover: world must be 1, 2, 4, 8 or 16");
    if (nbits < 2 * logW + 1) throw KgsError(KGS_E_ARG, "distributed prover: domain too small for the group (need n >= 2 W^2)");
    if (c.srs_power < 0) throw KgsError(KGS_E_ARG, "no SRS loaded");
    if (c.srs_power < nbits)
      throw KgsError(KGS_E_SRS, "The Powers of Tau file is not sufficiently large to commit the polynomials.");
    if (nbits > c.nbits_max) throw KgsError(KGS_E_SRS, "SRS loaded for a smaller maximum domain; reload with larger nbits_max");
    if (c.srs_slice_world > 1 && (c.srs_slice_world != W || c.srs_slice_rank != r))
      throw KgsError(KGS_E_ARG, "the loaded SRS slice (rank " + std::to_string(c.srs_slice_rank) + " of " +
                                    std::to_string(c.srs_slice_world) + ") is not this context's (rank " + std::to_string(r) +
                                    " of " + std::to_string(W) + ")");
    if (k < 1) throw KgsError(KGS_E_ARG, "The number of multisets must be greater than 0.");
    if (k > KGS_MAX_POLS) throw KgsError(KGS_E_ARG, "too many multisets");
    const uint64_t M = (1ull << nbits) / W;
    const int ncom_all = 2 * k + (in.sel_f ? 2 : 0) + 4;
    c.msm_slots = ncom_all + 4;
    c.ensure_pin(((size_t)ncom_all + 8) * ((size_t)c.tb.c * 128 + 64) +
                 32 * (size_t)((M + EVAL_TILE - 1) / EVAL_TILE) * (2 * k + 8) + ((size_t)kgs_ctx::SCAL_BYTES * 2) +
                 (8 << 20));
  } catch (const KgsError& e) {
    mine.code = e.code;
    snprintf(mine.msg, sizeof(mine.msg), "%s", e.what());
  } catch (const std::exception& e) {
    mine.code = KGS_E_HIP;
    snprintf(mine.msg, sizeof(mine.msg), "%s", e.what());
  }
  std::vector<Verdict> all(W);
  c.group->allgather(r, &mine, all.data(), sizeof(Verdict));
  for (int j = 0; j < W; j++)
    if (all[j].code != KGS_OK) {
      all[j].msg[sizeof(all[j].msg) - 1] = 0;
      throw KgsError(all[j].code, j == r ? std::string(all[j].msg)
                                         : std::string(all[j].msg) + " (on rank " + std::to_string(j) + ")");
    }
}

void prove_dist_impl(kgs_ctx& c, const ProveIn& in, uint8_t* com_out, uint8_t* ev_out) {
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  c.timing.resize(9, 0.0);
  for (int i = 0; i < 6; i++) c.timing[i] = 0.0;
  Range range(ROUND_NAMES[0]);
  auto lap = [&](int rr) {
    auto t1 = clk::now();
    c.timing[rr] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    t0 = t1;
    if (rr + 1 < 5) range.push(ROUND_NAMES[rr + 1]);
    else range.pop();
  };
  Dist D(c);
  const int W = D.W, r = D.r, logW = D.logW;
  const bool gs = in.kind != KGS_GRANDPRODUCT;  // KGS_LOOKUP is a selected grand-sum
  const bool lk = in.kind == KGS_LOOKUP;
  const bool sel = in.sel_f != nullptr;
  const int k = in.npols;
  const int nbits = in.nbits;
  const uint64_t n = 1ull << nbits;
  (void)logW;  // preconditions: dist_preconditions (decided by every rank together)
  const uint64_t M = n / W;  // local length of an n-vector in every layout
  const size_t EM = 32 * M;
  const int ncom_all = 2 * k + (sel ? 2 : 0) + 4;
  c.reset_staging();
  uint32_t* flags = c.buf("flags", 64);
  HC(hipMemsetAsync(flags, 0, 64, c.st));
  const bool vec = k > 1;
  const int slot0 = 0;
  int slot = slot0;

  // ---------------- round 1: witness polynomials + commitments (prover.js:144-179)
  std::vector<uint32_t*> fB(k), tB(k), Fc(k), Tc(k);
  uint32_t* eTmp = c.buf("d_eTmp", EM);
  for (int i = 0; i < k; i++) {
    fB[i] = c.buf("d_fB" + std::to_string(i), EM);
    tB[i] = c.buf("d_tB" + std::to_string(i), EM);
    Fc[i] = c.buf("d_Fc" + std::to_string(i), EM);
    Tc[i] = c.buf("d_Tc" + std::to_string(i), EM);
    launch_to_mont(c.st, fB[i], in.f_std[i] + (size_t)8 * r * M, M);
    launch_to_mont(c.st, tB[i], in.t_std[i] + (size_t)8 * r * M, M);
    launch_gather_e(c.st, eTmp, in.f_std[i], n, W, r, true);
    D.inv_e_to_cyc(Fc[i], eTmp, nbits, false);
    launch_gather_e(c.st, eTmp, in.t_std[i], n, W, r, true);
    D.inv_e_to_cyc(Tc[i], eTmp, nbits, false);
  }
  check_launch();
  // Montgomery write-back (prover.js:147-148): every rank returns the caller's full vectors
  bool wb = false;
  for (int i = 0; i < k; i++) wb |= !in.mont_f_out.empty() && (in.mont_f_out[i] || in.mont_t_out[i]);
  if (wb) {
    uint32_t* full = c.buf("d_wb", 32 * n);
    for (int i = 0; i < k; i++)
      for (int ft = 0; ft < 2; ft++) {
        uint8_t* dst = ft ? in.mont_t_out[i] : in.mont_f_out[i];
        if (!dst) continue;
        launch_to_mont(c.st, full, ft ? in.t_std[i] : in.f_std[i], n);
        HC(hipMemcpyAsync(dst, full, 32 * n, hipMemcpyDeviceToHost, c.st));
      }
  }
  const uint32_t *sFB = nullptr, *sTB = nullptr;
  uint32_t *sFc = nullptr, *sTc = nullptr;
  if (sel) {
    sFB = in.sel_f + (size_t)8 * r * M;
    sTB = in.sel_t + (size_t)8 * r * M;
    sFc = c.buf("d_sFc", EM);
    sTc = c.buf("d_sTc", EM);
    launch_gather_e(c.st, eTmp, in.sel_f, n, W, r, false);
    D.inv_e_to_cyc(sFc, eTmp, nbits, false);
    launch_gather_e(c.st, eTmp, in.sel_t, n, W, r, false);
    D.inv_e_to_cyc(sTc, eTmp, nbits, false);
  }
  // CYCLIC slice: scalar j of rank r multiplies SRS point r + W j
  auto commit_cyc = [&](const uint32_t* sc, uint64_t N) {
    const uint64_t cnt = N > (uint64_t)r ? (N - r + W - 1) / W : 0;
    return commit_launch_slice(c, sc, cnt, (uint64_t)r, (uint64_t)W, N, slot++, 0);
  };
  std::vector<Commit> r1;
  for (int i = 0; i < k; i++) {
    r1.push_back(commit_cyc(Fc[i], n));
    r1.push_back(commit_cyc(Tc[i], n));
  }
  if (sel) {
    r1.push_back(commit_cyc(sFc, n));
    r1.push_back(commit_cyc(sTc, n));
  }
  c.sync();
  if (in.after_round1) in.after_round1();
  std::vector<std::vector<uint8_t>> com(ncom_all, std::vector<uint8_t>(64));
  int ci = 0;
  {
    std::vector<uint8_t*> outs;
    for (size_t i = 0; i < r1.size(); i++) outs.push_back(com[ci++].data());
    commits_finish_with(c, r1, outs, W, D.host_ag());
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
  const uint32_t *fcomb = fB[0], *tcomb = tB[0], *polF = Fc[0], *polT = Tc[0];
  if (vec) {
    uint32_t* b_fe = c.buf("d_fcomb", EM);
    uint32_t* b_te = c.buf("d_tcomb", EM);
    uint32_t* b_F = c.buf("d_polF", EM);
    uint32_t* b_T = c.buf("d_polT", EM);
    LcTerms l1, l2, l3, l4;
    for (int i = 0; i < k; i++) {
      l1.add(fB[i], M, bpow[i]);
      l2.add(tB[i], M, bpow[i]);
      l3.add(Fc[i], M, bpow[i]);
      l4.add(Tc[i], M, bpow[i]);
    }
    run_lincomb(c.st, b_fe, M, l1);
    run_lincomb(c.st, b_te, M, l2);
    run_lincomb(c.st, b_F, M, l3);
    run_lincomb(c.st, b_T, M, l4);
    fcomb = b_fe;
    tcomb = b_te;
    polF = b_F;
    polT = b_T;
  }
  // builder on this rank's BLOCK of H (local scan), then the cross-rank offsets
  uint32_t* SB = c.buf("d_SB", EM);
  const uint32_t ntiles = (uint32_t)((M + EVAL_TILE - 1) / EVAL_TILE);
  uint32_t* d_gamma = c.scal(&gamma, 1);
  launch_builder(c.st, !gs, sel, SB, fcomb, tcomb, sFB, sTB, d_gamma, M, c.buf("bt_tp", 32 * (ntiles + 1)),
                 c.buf("bt_ti", 32 * (ntiles + 1)), flags + 8);  // flags[8]: the local wrap check, unused
  check_launch();
  uint8_t* h_tot = c.pin(32);
  HC(hipMemcpyAsync(h_tot, SB, 32, hipMemcpyDeviceToHost, c.st));  // SB[0] = local total
  HC(hipStreamSynchronize(c.st));
  const std::vector<Fr> tot = D.gather_fr({Fr::from_bytes(h_tot)});
  const Fr unit = gs ? Fr::zero() : Fr::one();
  Fr off = unit, all = unit, next = unit;
  for (int j = 0; j < W; j++) {
    if (j < r) off = gs ? off + tot[j] : off * tot[j];
    if (j <= r) next = gs ? next + tot[j] : next * tot[j];
    all = gs ? all + tot[j] : all * tot[j];
  }
  if (!(all == unit))  // S[0] = the total must be 0 (Z[0] = 1): grandsum.js:55-57, grandproduct.js:50-52
    throw KgsError(KGS_E_NOT_WELL_CALC, gs ? "The grand-sum polynomial S is not well calculated"
                                           : "The grand-product polynomial Z is not well calculated");
  if (r == W - 1) next = unit;  // S at the wrap (natural index n -> 0)
  Fr offs[2] = {off, next};
  uint32_t* d_offs = c.scal(offs, 2);
  launch_scan_fix(c.st, !gs, SB, d_offs, M);
  uint32_t* SE = c.buf("d_SE", EM);
  uint32_t* Sc = c.buf("d_Sc", EM);
  D.block_to_e(SE, SB, M);
  D.inv_e_to_cyc(Sc, SE, nbits, false);
  Commit cS = commit_cyc(Sc, n);
  // round 3's challenge-independent coset evaluations (E layout over the coset domain)
  const int lcs = (!gs && !sel) ? nbits : nbits + 1;
  const uint64_t cs = 1ull << lcs, Mc = cs / W;
  uint32_t* cosS = c.buf("d_cosS", 32 * Mc);
  uint32_t* cosF = c.buf("d_cosF", 32 * Mc);
  uint32_t* cosT = c.buf("d_cosT", 32 * Mc);
  uint32_t *cosSF = nullptr, *cosST = nullptr;
  D.fwd_cyc_to_e(cosS, Sc, M, lcs, true);
  D.fwd_cyc_to_e(cosF, polF, M, lcs, true);
  D.fwd_cyc_to_e(cosT, polT, M, lcs, true);
  if (sel) {
    cosSF = c.buf("d_cosSF", 32 * Mc);
    cosST = c.buf("d_cosST", 32 * Mc);
    D.fwd_cyc_to_e(cosSF, sFc, M, lcs, true);
    D.fwd_cyc_to_e(cosST, sTc, M, lcs, true);
  }
  // 1/(n (x_i - 1)) for this rank's coset points (cached per shape)
  const std::string nk = "d_nxm1_" + std::to_string(nbits) + "_" + std::to_string(lcs) + "_" + std::to_string(W) + "_" +
                         std::to_string(r);
  uint32_t* nxm1;
  if (c.dist_tabs.count(nk)) {
    nxm1 = c.dist_tabs[nk];
  } else {
    nxm1 = c.buf(nk, 32 * Mc);
    uint32_t* tmp = c.buf("d_nxm1_tmp", 32 * Mc);
    Fr kk[2] = {Fr::from_u64(5), Fr::from_u64(n)};
    uint32_t* d = c.scal(kk, 2);
    launch_nxm1_e(c.st, tmp, c.tw_fwd, lcs, d, d + 8, W, r);
    launch_fr_batch_inv(c.st, nxm1, tmp, Mc);
    check_launch();
    c.dist_tabs[nk] = nxm1;
  }
  c.sync();
  const int iS = ci;
  commits_finish_with(c, {cS}, {com[ci++].data()}, W, D.host_ag());
  lap(1);

  // ---------------- round 3: quotient on a coset (prover.js:233-286)
  tr.add_scalar(gamma);
  tr.add_commitment(com[iS].data());
  const Fr alpha = tr.challenge();
  const uint32_t rot = (uint32_t)(cs >> nbits);
  uint64_t qlen = (!gs && !sel) ? n - 1 : 2 * n - 2;  // deg Q + 1 bound
  Fr gn = Fr::from_u64(5).pow_u64(n);
  // alpha_t: weight of the selT-binary term (none for a lookup, whose selT holds multiplicities)
  Fr qs[5] = {alpha, gamma, (gn - Fr::one()).inverse(), (gn.neg() - Fr::one()).inverse(), lk ? Fr::zero() : alpha};
  uint32_t* d_qs = c.scal(qs, 5);
  // divisibility on H (BLOCK): S at the next natural index past this block is d_offs[1]
  launch_divcheck(c.st, !gs, sel, flags + 1, SB, fcomb, tcomb, sFB, sTB, d_qs, M, d_offs + 8, (uint64_t)r * M);
  // quotient halo: the first rot coset values of the chunk following each of this rank's blocks
  uint32_t* heads = c.buf("d_heads", 32 * 2 * W);
  launch_e_heads(c.st, heads, cosS, Mc, W, (int)rot);
  check_launch();
  uint8_t* h_heads = c.pin((size_t)32 * rot * W);
  HC(hipMemcpyAsync(h_heads, heads, (size_t)32 * rot * W, hipMemcpyDeviceToHost, c.st));
  HC(hipStreamSynchronize(c.st));
  std::vector<uint8_t> all_heads((size_t)32 * rot * W * W);
  D.allgather(h_heads, all_heads.data(), (size_t)32 * rot * W);
  uint8_t* h_halo = c.pin((size_t)32 * rot * W);
  for (int k1 = 0; k1 < W; k1++) {
    const int src = r + 1 < W ? r + 1 : 0;
    const int blk = r + 1 < W ? k1 : (k1 + 1) % W;
    memcpy(h_halo + (size_t)32 * rot * k1, all_heads.data() + (size_t)32 * rot * (W * src + blk), (size_t)32 * rot);
  }
  uint32_t* halo = c.buf("d_halo", 32 * 2 * W);
  HC(hipMemcpyAsync(halo, h_halo, (size_t)32 * rot * W, hipMemcpyHostToDevice, c.st));
  uint32_t* Qe = c.buf("d_Qe", 32 * Mc);
  uint32_t* Qc = c.buf("d_Qc", 32 * Mc);
  launch_quotient_e(c.st, !gs, sel, Qe, cosS, cosF, cosT, cosSF, cosST, nxm1, d_qs, halo, Mc, W, r, (int)rot);
  check_launch();
  D.inv_e_to_cyc(Qc, Qe, lcs, true);
  // Reference-quirks mode (ref_quirks.cpp; the single-GPU prover does the same in prover.cpp): where an
  // operand of degree 1 <= d < n/2 makes the reference's multiply compute something else (Q1), its
  // quotient chain is replayed on the gathered full operands, identically on every rank, and its Q —
  // or its error — replaces ours; otherwise only its RangeError on a zero quotient (Q3) differs.
  // Every decision here is made from all-gathered values, so all ranks throw the same error together.
  bool replayed = false;
  if (c.ref_quirks && !lk) {
    std::vector<const uint32_t*> ops = {polF, polT, Sc};
    if (sel) {
      ops.push_back(sFc);
      ops.push_back(sTc);
    }
    const std::vector<uint64_t> deg = D.degrees_cyc(ops, M);
    bool need = false;
    for (uint64_t d : deg) need |= d >= 1 && 2 * d < n;
    if (need) {
      // Only the replay's own decisions are the same on every rank (made from the gathered full
      // operands): its semantic errors (exempt in prove_dist_group anyway) and its "reference-quirks
      // mode:" refusals. A HIP or allocation failure in the gathers, the domain growth or the replay is
      // this rank's alone, stays un-agreed and aborts the group.
      const uint32_t* fF = D.gather_cyc(polF, M, "d_rq_F");
      const uint32_t* fT = D.gather_cyc(polT, M, "d_rq_T");
      const uint32_t* fS = D.gather_cyc(Sc, M, "d_rq_S");
      const uint32_t* fSF = sel ? D.gather_cyc(sFc, M, "d_rq_SF") : nullptr;
      const uint32_t* fST = sel ? D.gather_cyc(sTc, M, "d_rq_ST") : nullptr;
      uint32_t* fmut = nullptr;
      uint64_t qlen_ref = 0;
      const uint32_t* Qref = nullptr;
      try {
        Qref = ref_quirks_quotient(c, gs, sel, lk, nbits, alpha, gamma, fF, fT, fS, fSF, fST, qlen_ref, fmut);
      } catch (const KgsError& e) {
        if (e.code == KGS_E_ARG && e.what() && !strncmp(e.what(), "reference-quirks mode:", 22)) c.dist_err_agreed = true;
        throw;
      }
      if (fmut) {
        c.dist_err_agreed = true;
        throw KgsError(KGS_E_ARG, "reference-quirks mode: the replay wrote into polF's buffer (Q2); not reproduced by a rank group");
      }
      if (qlen_ref > cs) {
        c.dist_err_agreed = true;
        throw KgsError(KGS_E_ARG, "reference-quirks mode: the reference's Q has more coefficients than the group's coset layout");
      }
      // this rank's CYCLIC slice of the reference's Q (coefficients r + W j)
      HC(hipMemsetAsync(Qc, 0, 32 * Mc, c.st));
      const uint64_t cnt = qlen_ref > (uint64_t)r ? (qlen_ref - r + W - 1) / W : 0;
      if (cnt) HC(hipMemcpy2DAsync(Qc, 32, Qref + 8 * r, (size_t)32 * W, 32, cnt, hipMemcpyDeviceToDevice, c.st));
      qlen = qlen_ref;
      replayed = true;
    }
  }
  Commit cQ = commit_cyc(Qc, qlen);
  uint32_t* h_flags = (uint32_t*)c.pin(64);
  HC(hipMemcpyAsync(h_flags, flags, 64, hipMemcpyDeviceToHost, c.st));
  c.sync();
  if (!replayed) {
    if (D.gather_or(h_flags[1])) throw KgsError(KGS_E_NOT_DIVISIBLE, "Polynomial is not divisible");
    // Q3: the dividend of the reference's divZh has degree < n exactly when the quotient is zero
    // (degree 0 over all ranks: only global coefficient 0, rank 0's first, can still be nonzero)
    if (c.ref_quirks && !lk && D.degrees_cyc({Qc}, Mc)[0] == 0) {
      uint8_t* h0 = c.pin(32);
      HC(hipMemcpyAsync(h0, Qc, 32, hipMemcpyDeviceToHost, c.st));
      HC(hipStreamSynchronize(c.st));
      uint32_t nz = 0;
      for (int b = 0; b < 32; b++) nz |= h0[b];
      if (!D.gather_or(nz)) throw KgsError(KGS_E_RANGE, "offset is out of bounds");
    }
  }
  const int iQ = ci;
  commits_finish_with(c, {cQ}, {com[ci++].data()}, W, D.host_ag());
  lap(2);

  // ---------------- round 4: evaluations (prover.js:288-318): Horner on CYCLIC slices at x^W
  tr.add_scalar(alpha);
  tr.add_commitment(com[iQ].data());
  const Fr xi = tr.challenge();
  const Fr w = fr_w(nbits);
  const Fr xiw = xi * w;
  std::vector<const uint32_t*> esrc;
  std::vector<uint64_t> elen;
  for (int i = 0; i < k; i++) {
    esrc.push_back(Fc[i]);
    elen.push_back(M);
    if (gs) {
      esrc.push_back(Tc[i]);
      elen.push_back(M);
    }
  }
  if (sel) {
    esrc.push_back(sFc);
    elen.push_back(M);
    esrc.push_back(sTc);
    elen.push_back(M);
  }
  EvalJob ej1 = eval_launch(c, esrc, elen, xi.pow_u64((uint64_t)W), 0);
  EvalJob ej2 = eval_launch(c, {Sc}, {M}, xiw.pow_u64((uint64_t)W), 1);
  c.sync();
  std::vector<Fr> loc = eval_finish(ej1);
  loc.push_back(eval_finish(ej2)[0]);
  const std::vector<Fr> allv = D.gather_fr(loc);
  const size_t np = loc.size();
  std::vector<Fr> ev1(np - 1, Fr::zero());
  Fr sxiw = Fr::zero();
  {
    Fr xr = Fr::one(), xwr = Fr::one();
    for (int j = 0; j < W; j++) {
      for (size_t p = 0; p + 1 < np; p++) ev1[p] = ev1[p] + xr * allv[j * np + p];
      sxiw = sxiw + xwr * allv[j * np + np - 1];
      xr = xr * xi;
      xwr = xwr * xiw;
    }
  }
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
  const R5 r5 = round5_terms(gs, sel, k, nbits, alpha, beta, gamma, v, xi, fx, tx, sFx, sTx, sxiw, lk);
  const uint64_t qcnt = qlen > (uint64_t)r ? (qlen - r + W - 1) / W : 0;
  LcTerms lw;
  for (const R5Term& t : r5.terms) {
    switch (t.id) {
      case R5_S: lw.add(Sc, M, t.coef); break;
      case R5_Q: lw.add(Qc, qcnt, t.coef); break;
      case R5_F: lw.add(Fc[t.idx], M, t.coef); break;
      case R5_T: lw.add(Tc[t.idx], M, t.coef); break;
      case R5_SELF: lw.add(sFc, M, t.coef); break;
      case R5_SELT: lw.add(sTc, M, t.coef); break;
      case R5_POLT: lw.add(polT, M, t.coef); break;
    }
  }
  lw.c0 = r == 0 ? r5.c0 : Fr::zero();  // the constant term lives at global index 0 (rank 0)
  const uint64_t L = qlen > n ? qlen : n;
  // numerator P (CYCLIC over cs >= L points) -> BLOCK -> division by (X - xi) with carries
  uint32_t* Pc = c.buf("d_Pc", 32 * Mc);
  uint32_t* PB = c.buf("d_PB", 32 * Mc);
  uint32_t* WxB = c.buf("d_WxB", 32 * Mc);
  run_lincomb(c.st, Pc, Mc, lw);
  D.cyc_to_block(PB, Pc, Mc);
  const uint32_t dt1 = (uint32_t)((Mc + EVAL_TILE - 1) / EVAL_TILE);
  launch_divide(c.st, WxB, flags + 9, PB, Mc, xpowers(c, xi), c.buf("div_part", 32 * (dt1 + 1)),
                c.buf("div_carry", 32 * (dt1 + 1)));
  EvalJob eR1 = eval_launch(c, {PB}, {Mc}, xi, 2);  // R_lo: this block's value at xi with zero carry-in
  // W_{xi w}: (S - S(xi w)) (CYCLIC over n) -> BLOCK -> division by (X - xi w)
  LcTerms l2;
  l2.add(Sc, M, Fr::one());
  l2.c0 = r == 0 ? sxiw.neg() : Fr::zero();
  uint32_t* P2c = c.buf("d_P2c", EM);
  uint32_t* P2B = c.buf("d_P2B", EM);
  uint32_t* W2B = c.buf("d_W2B", EM);
  run_lincomb(c.st, P2c, M, l2);
  D.cyc_to_block(P2B, P2c, M);
  launch_divide(c.st, W2B, flags + 10, P2B, M, xpowers(c, xiw), c.buf("div_part2", 32 * (ntiles + 1)),
                c.buf("div_carry2", 32 * (ntiles + 1)));
  EvalJob eR2 = eval_launch(c, {P2B}, {M}, xiw, 3);
  c.sync();
  const std::vector<Fr> Rl = D.gather_fr({eval_finish(eR1)[0], eval_finish(eR2)[0]});
  // carries from the top rank down: c_{W-1} = 0, c_{j-1} = R_lo(j) + z^len c_j; remainder at rank 0
  auto carries = [&](int which, const Fr& z, uint64_t len, Fr& mine) {
    const Fr zl = z.pow_u64(len);
    Fr cr = Fr::zero();
    for (int j = W - 1; j >= 0; j--) {
      if (j == r) mine = cr;
      cr = Rl[2 * j + which] + zl * cr;
    }
    return cr;  // r_0: must be zero
  };
  Fr c1, c2;
  const bool bad1 = !carries(0, xi, Mc, c1).is_zero();
  const bool bad2 = !carries(1, xiw, M, c2).is_zero();
  if (bad1 || bad2) throw KgsError(KGS_E_DOES_NOT_DIVIDE, "Polynomial does not divide");
  Fr cc[2] = {c1, c2};
  uint32_t* d_cc = c.scal(cc, 2);
  uint32_t* pz1 = c.buf("d_pz1", 32 * Mc);
  uint32_t* pz2 = c.buf("d_pz2", EM);
  Fr zz[2] = {xi, xiw};
  uint32_t* d_zz = c.scal(zz, 2);
  launch_powers(c.st, pz1, Mc, d_zz, nullptr);
  launch_powers(c.st, pz2, M, d_zz + 8, nullptr);
  launch_div_fix(c.st, WxB, pz1, d_cc, Mc);
  launch_div_fix(c.st, W2B, pz2, d_cc + 8, M);
  check_launch();
  // the openings go back to CYCLIC (one all-to-all each), so that every MSM of the proof reads the
  // same per-rank SRS slice (points r + W j: kgs_srs_load_ptau_slice)
  uint32_t* WxC = c.buf("d_WxC", 32 * Mc);
  uint32_t* W2C = c.buf("d_W2C", EM);
  D.block_to_cyc(WxC, WxB, Mc);
  D.block_to_cyc(W2C, W2B, M);
  Commit cW1 = commit_cyc(WxC, L - 1);
  Commit cW2 = commit_cyc(W2C, n - 1);
  c.sync();
  commits_finish_with(c, {cW1, cW2}, {com[ci].data(), com[ci + 1].data()}, W, D.host_ag());
  ci += 2;
  lap(4);

  for (int i = 0; i < ncom_all; i++) memcpy(com_out + 64 * i, com[i].data(), 64);
  for (size_t i = 0; i < evals.size(); i++) evals[i].to_bytes(ev_out + 32 * i);
  c.reset_staging();
  D.finish_stats();
}

// Preconditions are agreed by all ranks (dist_preconditions: they all throw together, the group
// stays usable); semantic failures (decided from all-gathered values: the same on every rank) leave
// the group usable too; anything else happened on this rank alone mid-proof and aborts the group, so
// that the other ranks fail at their next exchange instead of waiting in it (RCCL: at the
// KGS_GROUP_TIMEOUT_S deadline of RcclGroup::wait).
extern thread_local int tl_group_rank;  // prover.cpp dev_malloc: per-rank fault injection
void prove_dist_group(kgs_ctx& c, const ProveIn& in, uint8_t* com_out, uint8_t* ev_out) {
  c.xs.reset();
  c.dist_err_agreed = false;
  struct RankTag {
    int prev;
    explicit RankTag(int r) : prev(tl_group_rank) { tl_group_rank = r; }
    ~RankTag() { tl_group_rank = prev; }
  } tag(c.group_rank);
  dist_preconditions(c, in);
  try {
    prove_dist_impl(c, in, com_out, ev_out);
  } catch (const KgsError& e) {
    if (e.code != KGS_E_NOT_WELL_CALC && e.code != KGS_E_NOT_DIVISIBLE && e.code != KGS_E_DOES_NOT_DIVIDE &&
        e.code != KGS_E_RANGE && !c.dist_err_agreed)
      c.group->abort();
    throw;
  } catch (...) {
    c.group->abort();
    throw;
  }
}

}  // namespace kgsi

// ================================================================== C-ABI
#define API_BEGIN try {
#define API_END                               \
  }                                           \
  catch (const KgsError& e) {                 \
    return kgs_fail(e);                       \
  }                                           \
  catch (const std::exception& e) {           \
    kgs_errbuf() = e.what();                  \
    return KGS_E_HIP;                         \
  }                                           \
  return KGS_OK;

static void check_world(int world) {
  if (world < 1 || world > 16 || (world & (world - 1))) throw KgsError(KGS_E_ARG, "group world must be 1, 2, 4, 8 or 16");
}

extern "C" {

int kgs_group_create_local(int world, kgs_group_t** out) {
  API_BEGIN
  if (!out) throw KgsError(KGS_E_ARG, "NULL argument");
  check_world(world);
  *out = new LocalGroup(world);
  API_END
}

int kgs_group_create_host(int world, kgs_allgather_fn fn, void* user, kgs_group_t** out) {
  API_BEGIN
  if (!out || !fn) throw KgsError(KGS_E_ARG, "NULL argument");
  check_world(world);
  *out = new HostGroup(world, fn, nullptr, user);
  API_END
}

int kgs_group_create_host_a2a(int world, kgs_allgather_fn fn, kgs_alltoall_fn a2a, void* user, kgs_group_t** out) {
  API_BEGIN
  if (!out || !fn || !a2a) throw KgsError(KGS_E_ARG, "NULL argument");
  check_world(world);
  *out = new HostGroup(world, fn, a2a, user);
  API_END
}

int kgs_last_exchange(kgs_ctx_t* ctx, double* out, int max) {
  if (!ctx || !out) return KGS_E_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  const ExchangeStats& x = ctx->xs;
  const double v[6] = {(double)x.a2a_n, x.a2a_ms, (double)x.a2a_bytes, (double)x.ag_n, x.ag_ms, (double)x.ag_bytes};
  const int n = max < 6 ? max : 6;
  for (int i = 0; i < n; i++) out[i] = v[i];
  return n;
}

int kgs_group_rccl_unique_id(uint8_t id[128]) {
  API_BEGIN
  if (!id) throw KgsError(KGS_E_ARG, "NULL argument");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId u;
  NC(ncclGetUniqueId(&u));
  memcpy(id, &u, 128);
  API_END
}

int kgs_group_create_rccl(int rank, int world, const uint8_t id[128], int device, kgs_group_t** out) {
  API_BEGIN
  if (!out || !id) throw KgsError(KGS_E_ARG, "NULL argument");
  check_world(world);
  if (rank < 0 || rank >= world) throw KgsError(KGS_E_ARG, "bad rank");
  HC(hipSetDevice(device));
  auto* g = new RcclGroup();
  g->world = world;
  g->device = device;
  try {
    HC(hipStreamCreateWithFlags(&g->st_small, hipStreamNonBlocking));
    ncclUniqueId u;
    memcpy(&u, id, 128);
    NC(ncclCommInitRank(&g->comm, world, u, rank));
  } catch (...) {
    delete g;
    throw;
  }
  *out = g;
  API_END
}

void kgs_group_destroy(kgs_group_t* g) { delete g; }

int kgs_group_world(kgs_group_t* g, int* world) {
  if (!g || !world) return KGS_E_ARG;
  *world = g->world;
  return KGS_OK;
}

int kgs_ctx_set_group(kgs_ctx_t* ctx, kgs_group_t* g, int rank) {
  API_BEGIN
  if (!ctx) throw KgsError(KGS_E_ARG, "NULL ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (g && (rank < 0 || rank >= g->world)) throw KgsError(KGS_E_ARG, "bad rank for this group");
  if (g) g->attach(rank, ctx->device);
  ctx->group = g;  // a world-1 group runs the distributed code path on one rank (transport check)
  ctx->group_rank = ctx->group ? rank : 0;
  API_END
}

}  // extern "C"
