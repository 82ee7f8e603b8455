// N-API addon (Node >= 12, N-API 8) binding the C-ABI of libkgs.so (include/kgs.h) for the
// JavaScript drop-in modules in js/src. Heavy calls (SRS load, prove) run in napi_async_work and
// return Promises, like the reference's async module API.
#include <node_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <map>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kgs.h"

#define NAPI_CALL(env, call)                                        \
  do {                                                              \
    if ((call) != napi_ok) {                                        \
      napi_throw_error((env), nullptr, "N-API call failed: " #call); \
      return nullptr;                                               \
    }                                                               \
  } while (0)

static kgs_ctx_t* get_ctx(napi_env env, napi_value v) {
  void* p = nullptr;
  napi_get_value_external(env, v, &p);
  return (kgs_ctx_t*)p;
}

static std::vector<uint8_t> bytes_of(napi_env env, napi_value v) {
  std::vector<uint8_t> out;
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (is_ta) {
    napi_typedarray_type t;
    size_t len;
    void* data;
    napi_value ab;
    size_t off;
    napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off);
    out.assign((uint8_t*)data, (uint8_t*)data + len);
    return out;
  }
  bool is_buf = false;
  napi_is_buffer(env, v, &is_buf);
  if (is_buf) {
    void* data;
    size_t len;
    napi_get_buffer_info(env, v, &data, &len);
    out.assign((uint8_t*)data, (uint8_t*)data + len);
  }
  return out;
}

// zero-copy view of a Uint8Array / Buffer argument, kept alive by a reference until the async
// work completes (ArrayBuffer backing stores do not move)
struct View {
  const uint8_t* p = nullptr;
  size_t len = 0;
};
static View view_of(napi_env env, napi_value v, std::vector<napi_ref>& refs) {
  View out;
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (is_ta) {
    napi_typedarray_type t;
    size_t len;
    void* data;
    napi_value ab;
    size_t off;
    napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off);
    out.p = (const uint8_t*)data;
    out.len = len;
  } else {
    bool is_buf = false;
    napi_is_buffer(env, v, &is_buf);
    if (is_buf) {
      void* data;
      size_t len;
      napi_get_buffer_info(env, v, &data, &len);
      out.p = (const uint8_t*)data;
      out.len = len;
    }
  }
  napi_ref r;
  if (napi_create_reference(env, v, 1, &r) == napi_ok) refs.push_back(r);
  return out;
}

// Output buffers handed to JS (the Montgomery forms the reference writes back into the caller's
// Evaluations, prover.js:147-148): 64 MiB per proof at n = 2^20. Fresh malloc'd memory costs a page
// fault per 4 KiB (16 K per buffer) on first touch and an munmap on release, which under several
// concurrent proofs serialise on the process's memory map. So: 2 MiB-aligned anonymous mappings
// with MADV_HUGEPAGE (32x fewer faults where transparent huge pages are enabled), recycled through a
// free list when the JS garbage collector releases them (up to 2 GiB cached), and reported to V8 as
// external memory so that collection keeps pace with the proofs.
namespace {
std::mutex g_out_mu;
std::multimap<size_t, void*> g_out_free;
size_t g_out_cached = 0;
constexpr size_t OUT_CACHE_MAX = (size_t)2 << 30;
constexpr size_t HUGE = (size_t)2 << 20;

size_t out_round(size_t len) { return (len + HUGE - 1) / HUGE * HUGE; }

// KGS_JS_OUT_REGISTER=1: pin every output buffer for its life so the write-back is DMA'd in place.
// Off by default: registering a fresh 32 MiB buffer inside the call costs more than the staging copy
// it saves whenever the caller keeps its outputs (profiles/r03/boundary_ab.txt, profiles/r04/js/). A pool
// of pre-registered, pre-faulted spares topped up by a background thread was tried too (round 4):
// no faster, and the thread's registrations kept the process from exiting.
bool out_registered() {
  static const bool reg = getenv("KGS_JS_OUT_REGISTER") != nullptr;
  return reg;
}

uint8_t* out_map(size_t sz) {
  // over-allocate by one huge page to align the start, then trim the ends
  void* raw = mmap(nullptr, sz + HUGE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (raw == MAP_FAILED) return nullptr;
  uintptr_t a = ((uintptr_t)raw + HUGE - 1) & ~(uintptr_t)(HUGE - 1);
  if (a > (uintptr_t)raw) munmap(raw, a - (uintptr_t)raw);
  const uintptr_t end = (uintptr_t)raw + sz + HUGE;
  if (end > a + sz) munmap((void*)(a + sz), end - (a + sz));
  madvise((void*)a, sz, MADV_HUGEPAGE);
  if (out_registered() && kgs_host_register((void*)a, sz) != KGS_OK) {
    munmap((void*)a, sz);
    return nullptr;
  }
  return (uint8_t*)a;
}

uint8_t* out_alloc(size_t len) {
  const size_t sz = out_round(len);
  {
    std::lock_guard<std::mutex> lk(g_out_mu);
    auto it = g_out_free.find(sz);
    if (it != g_out_free.end()) {
      void* p = it->second;
      g_out_free.erase(it);
      g_out_cached -= sz;
      return (uint8_t*)p;
    }
  }
  return out_map(sz);
}

void out_release(uint8_t* p, size_t len) {
  const size_t sz = out_round(len);
  {
    std::lock_guard<std::mutex> lk(g_out_mu);
    if (g_out_cached + sz <= OUT_CACHE_MAX) {
      g_out_free.emplace(sz, p);
      g_out_cached += sz;
      return;
    }
  }
  if (out_registered()) kgs_host_unregister(p);
  munmap(p, sz);
}
}  // namespace


// External memory adopted by JS but not yet reported to V8. Reporting it (napi_adjust_external_memory)
// can start a full GC right there; done in the completion callback, that GC ran before the proof's
// Promise resolved (+6 ms per proof at n = 2^20). It is reported when the next proof has been
// queued instead (flush_external), so the GC overlaps that proof's GPU work. Main thread only.
static int64_t g_ext_pending = 0;
static void flush_external(napi_env env) {
  if (g_ext_pending > 0) {
    int64_t adj = 0;
    napi_adjust_external_memory(env, g_ext_pending, &adj);
    g_ext_pending = 0;
  }
}

static void out_finalize(napi_env env, void* data, void* hint) {
  const int64_t len = (int64_t)(uintptr_t)hint;
  if (g_ext_pending >= len) {
    g_ext_pending -= len;  // not reported yet
  } else {
    int64_t adj = 0;
    napi_adjust_external_memory(env, -len, &adj);
  }
  out_release((uint8_t*)data, (size_t)len);
}

// Uint8Array over an out_alloc'd buffer handed to JS without a copy (recycled by the GC finalizer)
static napi_value adopt_u8(napi_env env, uint8_t* data, size_t len) {
  napi_value ab, ta;
  if (napi_create_external_arraybuffer(env, data, len, out_finalize, (void*)(uintptr_t)len, &ab) != napi_ok) {
    out_release(data, len);
    return nullptr;
  }
  g_ext_pending += (int64_t)len;
  napi_create_typedarray(env, napi_uint8_array, len, ab, 0, &ta);
  return ta;
}

static napi_value make_u8(napi_env env, const uint8_t* data, size_t len) {
  void* buf;
  napi_value ab, ta;
  napi_create_arraybuffer(env, len, &buf, &ab);
  memcpy(buf, data, len);
  napi_create_typedarray(env, napi_uint8_array, len, ab, 0, &ta);
  return ta;
}

static void ctx_finalize(napi_env, void* data, void*) { kgs_ctx_destroy((kgs_ctx_t*)data); }

// ctxCreate(device) -> External
static napi_value CtxCreate(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  int32_t dev = 0;
  if (argc > 0) napi_get_value_int32(env, argv[0], &dev);
  kgs_ctx_t* ctx = nullptr;
  if (kgs_ctx_create(dev, &ctx) != KGS_OK) {
    napi_throw_error(env, nullptr, kgs_last_error());
    return nullptr;
  }
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, ctx, ctx_finalize, nullptr, &ext));
  return ext;
}

// deviceCount() -> number of visible HIP devices
static napi_value DeviceCount(napi_env env, napi_callback_info) {
  int n = 0;
  if (kgs_device_count(&n) != KGS_OK) {
    napi_throw_error(env, nullptr, kgs_last_error());
    return nullptr;
  }
  napi_value v;
  napi_create_int32(env, n, &v);
  return v;
}

// ptauPower(path) -> power from the ptau header (readPTauHeader, src/ptau_utils.js:3-24)
static napi_value PtauPower(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  size_t len = 0;
  napi_get_value_string_utf8(env, argv[0], nullptr, 0, &len);
  std::string path(len + 1, '\0');
  napi_get_value_string_utf8(env, argv[0], &path[0], len + 1, &len);
  path.resize(len);
  int power = 0;
  if (kgs_ptau_power(path.c_str(), &power) != KGS_OK) {
    napi_throw_error(env, nullptr, kgs_last_error());
    return nullptr;
  }
  napi_value v;
  napi_create_int32(env, power, &v);
  return v;
}

// keccak256(Uint8Array) -> Uint8Array(32)
static napi_value Keccak(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  std::vector<uint8_t> d = bytes_of(env, argv[0]);
  uint8_t out[32];
  kgs_keccak256(d.data(), d.size(), out);
  return make_u8(env, out, 32);
}

// srsInfo(ctx) -> {power, npts, windowC}
static napi_value SrsInfo(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  int power = 0, c = 0;
  uint64_t npts = 0;
  if (kgs_srs_info(get_ctx(env, argv[0]), &power, &npts, &c) != KGS_OK) {
    napi_throw_error(env, nullptr, kgs_last_error());
    return nullptr;
  }
  napi_value o, v;
  napi_create_object(env, &o);
  napi_create_int32(env, power, &v);
  napi_set_named_property(env, o, "power", v);
  napi_create_double(env, (double)npts, &v);
  napi_set_named_property(env, o, "npts", v);
  napi_create_int32(env, c, &v);
  napi_set_named_property(env, o, "windowC", v);
  return o;
}

// ---------------------------------------------------------------- async work
struct Job {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  kgs_ctx_t* ctx = nullptr;
  int op = 0;  // 0 = load ptau, 1 = prove, 2 = elementwise Fr map / transform (frOp),
               // 3 = one distributed proof over a rank group (proveGroup), 4 = msmPoints
  int rc = 0;
  std::string err;
  // load
  std::string path;
  int nbits_max = -1;
  // prove
  int kind = 0, nbits = 0, npols = 0;
  std::vector<View> f, t;
  View sf, st;
  std::vector<uint8_t*> mf, mt;  // malloc'd, adopted by JS on success
  std::vector<uint8_t> com, ev;
  std::vector<napi_ref> refs;
  bool selected = false;
  bool want_mont = true;  // false: no Montgomery write-back (the other ranks of a distributed proof)
  double exec_ms = 0;     // wall time of job_execute (the libkgs call on the worker thread)
  // diagnostics: queued (main thread) -> execute start / end (libuv worker) -> complete (main thread)
  std::chrono::steady_clock::time_point t_queue, t_exec0, t_exec1;
  // proveGroup: rank r's context, SRS slice r of W, one native thread per rank
  std::vector<kgs_ctx_t*> ranks;
  // msmPoints: bases and standard-form scalars (copied: the call returns before the work runs)
  std::vector<uint8_t> bases, scal;
  uint8_t msm_out[64];
  // frOp
  int fr_op = 0;
  View in;
  uint8_t* out = nullptr;  // out_alloc'd, adopted by JS on success
  size_t out_len = 0;
};

static void prove_one(Job* j, kgs_ctx_t* ctx, bool mont, std::vector<uint8_t>& com, std::vector<uint8_t>& ev, int& rc,
                      std::string& err) {
  int nc = 0, ne = 0;
  kgs_proof_shape(j->kind, j->npols, j->selected ? 1 : 0, &nc, &ne);
  com.resize(64 * (size_t)nc);
  ev.resize(32 * (size_t)ne);
  std::vector<const uint8_t*> fp, tp;
  for (int i = 0; i < j->npols; i++) {
    fp.push_back(j->f[i].p);
    tp.push_back(j->t[i].p);
  }
  rc = kgs_prove(ctx, j->kind, j->nbits, j->npols, fp.data(), tp.data(), j->selected ? j->sf.p : nullptr,
                 j->selected ? j->st.p : nullptr, mont ? j->mf.data() : nullptr, mont ? j->mt.data() : nullptr,
                 com.data(), ev.data());
  if (rc != KGS_OK) err = kgs_last_error();
}

// the inputs' shape, and (want_mont) the output buffers of the Montgomery write-back
static bool prepare_prove(Job* j) {
  const size_t E = (size_t)32 << j->nbits;
  bool ok = true;
  for (int i = 0; i < j->npols; i++) {
    ok &= j->f[i].len == E && j->t[i].len == E;
    if (j->want_mont) {
      j->mf.push_back(out_alloc(E));
      j->mt.push_back(out_alloc(E));
      ok &= j->mf.back() && j->mt.back();
    }
  }
  if (j->selected) ok &= j->sf.len == E && j->st.len == E;
  if (!ok) {
    j->rc = KGS_E_ARG;
    j->err = "evaluation buffers must hold 2^nbits 32-byte elements";
  }
  return ok;
}

// One distributed proof: every rank on its own native thread (the group's barriers join them), so
// the ranks never compete with each other — or with the context pool's proofs — for libuv's
// thread pool (a rank waiting at a barrier for a rank that never got a pool thread would stall).
// Each rank first makes its SRS slice resident (kgs_srs_load_ptau_slice: points r + W j), then
// proves; rank 0 returns the proof and the Montgomery write-back, every rank's proof must agree.
static void group_execute(Job* j) {
  const int W = (int)j->ranks.size();
  std::vector<int> rc(W, KGS_OK);
  std::vector<std::string> err(W);
  std::vector<std::vector<uint8_t>> com(W), ev(W);
  std::vector<std::thread> th;
  for (int r = 0; r < W; r++)
    th.emplace_back([&, r] {
      rc[r] = kgs_srs_load_ptau_slice(j->ranks[r], j->path.c_str(), j->nbits, r, W);
      if (rc[r] != KGS_OK) err[r] = kgs_last_error();
      // a rank whose load failed still enters the prover: the group agrees on the failure there
      int rp = KGS_OK;
      std::string ep;
      prove_one(j, j->ranks[r], r == 0 && j->want_mont, com[r], ev[r], rp, ep);
      if (rc[r] == KGS_OK) {
        rc[r] = rp;
        err[r] = ep;
      }
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < W; r++)
    if (rc[r] != KGS_OK) {
      j->rc = rc[r];
      j->err = err[r];
      return;
    }
  for (int r = 1; r < W; r++)
    if (com[r] != com[0] || ev[r] != ev[0]) {
      j->rc = KGS_E_COMM;
      j->err = "ranks of the distributed proof disagree";
      return;
    }
  j->com = com[0];
  j->ev = ev[0];
}

static void job_execute(napi_env, void* data) {
  Job* j = (Job*)data;
  const auto t0 = std::chrono::steady_clock::now();
  j->t_exec0 = t0;
  struct Stamp {
    Job* j;
    std::chrono::steady_clock::time_point t0;
    ~Stamp() {
      j->t_exec1 = std::chrono::steady_clock::now();
      j->exec_ms = std::chrono::duration<double, std::milli>(j->t_exec1 - t0).count();
    }
  } stamp{j, t0};
  if (j->op == 0) {
    j->rc = kgs_srs_load_ptau(j->ctx, j->path.c_str(), j->nbits_max);
  } else if (j->op == 2) {
    const uint64_t n = j->in.len / 32;
    j->out_len = j->in.len;
    j->out = out_alloc(j->out_len);
    if (!j->out) {
      j->rc = KGS_E_ARG;
      j->err = "out of host memory";
      return;
    }
    int logm = 0;
    while ((1ull << logm) < n) logm++;
    switch (j->fr_op) {
      case 0: j->rc = kgs_fr_to_mont(j->ctx, j->in.p, j->out, n); break;
      case 1: j->rc = kgs_fr_from_mont(j->ctx, j->in.p, j->out, n); break;
      case 2: j->rc = kgs_fr_batch_inverse(j->ctx, j->in.p, j->out, n); break;
      default: j->rc = kgs_ntt(j->ctx, j->in.p, j->out, logm, j->fr_op == 4); break;
    }
  } else if (j->op == 3) {
    if (prepare_prove(j)) group_execute(j);
    return;
  } else if (j->op == 4) {
    const uint64_t n = j->scal.size() / 32;
    int lg = 0;
    while ((1ull << (lg + 1)) < n) lg++;
    std::vector<uint8_t> mont(j->scal.size());
    j->rc = kgs_srs_load_points(j->ctx, j->bases.data(), n, lg, lg);
    if (j->rc == KGS_OK) j->rc = kgs_fr_to_mont(j->ctx, j->scal.data(), mont.data(), n);
    if (j->rc == KGS_OK) j->rc = kgs_msm(j->ctx, mont.data(), n, j->msm_out);
  } else {
    if (!prepare_prove(j)) return;
    std::string e;
    prove_one(j, j->ctx, j->want_mont, j->com, j->ev, j->rc, e);
    if (j->rc != KGS_OK) j->err = e;
    return;
  }
  if (j->rc != KGS_OK) j->err = kgs_last_error();
}

static void job_complete(napi_env env, napi_status, void* data) {
  Job* j = (Job*)data;
  if (j->rc != KGS_OK) {
    napi_value msg, err, code;
    napi_create_string_utf8(env, j->err.c_str(), NAPI_AUTO_LENGTH, &msg);
    // the reference's divZh on a zero quotient throws V8's RangeError (reference-quirks mode only)
    if (j->rc == KGS_E_RANGE) napi_create_range_error(env, nullptr, msg, &err);
    else napi_create_error(env, nullptr, msg, &err);
    napi_create_int32(env, j->rc, &code);
    napi_set_named_property(env, err, "kgsCode", code);
    napi_reject_deferred(env, j->deferred, err);
  } else if (j->op == 0) {
    napi_value u;
    napi_get_undefined(env, &u);
    napi_resolve_deferred(env, j->deferred, u);
  } else if (j->op == 2) {
    napi_resolve_deferred(env, j->deferred, adopt_u8(env, j->out, j->out_len));
    j->out = nullptr;
  } else if (j->op == 4) {
    napi_resolve_deferred(env, j->deferred, make_u8(env, j->msm_out, 64));
  } else {
    napi_value o, arr;
    napi_create_object(env, &o);
    napi_create_array(env, &arr);
    for (size_t i = 0; i < j->com.size() / 64; i++) napi_set_element(env, arr, (uint32_t)i, make_u8(env, &j->com[64 * i], 64));
    napi_set_named_property(env, o, "commitments", arr);
    napi_create_array(env, &arr);
    for (size_t i = 0; i < j->ev.size() / 32; i++) napi_set_element(env, arr, (uint32_t)i, make_u8(env, &j->ev[32 * i], 32));
    napi_set_named_property(env, o, "evaluations", arr);
    napi_create_array(env, &arr);
    const size_t E = (size_t)32 << j->nbits;
    for (size_t i = 0; i < j->mf.size(); i++) napi_set_element(env, arr, (uint32_t)i, adopt_u8(env, j->mf[i], E));
    napi_set_named_property(env, o, "montF", arr);
    napi_create_array(env, &arr);
    for (size_t i = 0; i < j->mt.size(); i++) napi_set_element(env, arr, (uint32_t)i, adopt_u8(env, j->mt[i], E));
    napi_set_named_property(env, o, "montT", arr);
    napi_value ems;
    napi_create_double(env, j->exec_ms, &ems);
    napi_set_named_property(env, o, "execMs", ems);  // diagnostics: time inside libkgs
    // diagnostics: [queued -> worker start, worker end -> this completion callback] in ms
    const auto tc = std::chrono::steady_clock::now();
    napi_create_array(env, &arr);
    const double d0 = std::chrono::duration<double, std::milli>(j->t_exec0 - j->t_queue).count();
    const double d1 = std::chrono::duration<double, std::milli>(tc - j->t_exec1).count();
    napi_create_double(env, d0, &ems);
    napi_set_element(env, arr, 0, ems);
    napi_create_double(env, d1, &ems);
    napi_set_element(env, arr, 1, ems);
    napi_set_named_property(env, o, "waitMs", arr);
    j->mf.clear();
    j->mt.clear();
    napi_resolve_deferred(env, j->deferred, o);
  }
  const size_t Eo = (size_t)32 << j->nbits;
  for (uint8_t* p : j->mf)  // error path: not adopted
    if (p) out_release(p, Eo);
  for (uint8_t* p : j->mt)
    if (p) out_release(p, Eo);
  if (j->out) out_release(j->out, j->out_len);
  for (napi_ref r : j->refs) napi_delete_reference(env, r);
  napi_delete_async_work(env, j->work);
  delete j;
}

static napi_value queue(napi_env env, Job* j, const char* name) {
  napi_value promise, rname;
  NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
  napi_create_string_utf8(env, name, NAPI_AUTO_LENGTH, &rname);
  NAPI_CALL(env, napi_create_async_work(env, nullptr, rname, job_execute, job_complete, j, &j->work));
  j->t_queue = std::chrono::steady_clock::now();
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  if (j->op == 1 || j->op == 3) flush_external(env);  // a GC it starts now runs beside the proof just queued
  return promise;
}

// srsLoadPtau(ctx, path, nbitsMax) -> Promise<void>
static napi_value SrsLoad(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Job* j = new Job();
  j->op = 0;
  j->ctx = get_ctx(env, argv[0]);
  size_t len;
  napi_get_value_string_utf8(env, argv[1], nullptr, 0, &len);
  j->path.resize(len + 1);
  napi_get_value_string_utf8(env, argv[1], &j->path[0], len + 1, &len);
  j->path.resize(len);
  if (argc > 2) napi_get_value_int32(env, argv[2], &j->nbits_max);
  return queue(env, j, "kgs_srs_load");
}

// prove(ctx, kind, nbits, [F...], [T...], selF|null, selT|null[, wantMont = true])
//   -> Promise<{commitments, evaluations, montF, montT}> (montF/montT empty without wantMont)
static napi_value prove_args(napi_env env, napi_value* argv, size_t argc, Job* j);
static napi_value Prove(napi_env env, napi_callback_info info) {
  size_t argc = 8;
  napi_value argv[8];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Job* j = new Job();
  j->op = 1;
  j->ctx = get_ctx(env, argv[0]);
  return prove_args(env, argv, argc, j);
}

// proveGroup([ctx_0..ctx_{W-1}], ptauPath, kind, nbits, [F...], [T...], selF|null, selT|null)
//   -> Promise<{commitments, evaluations, montF, montT}>: one proof over the contexts' rank group
//   (ctxSetGroup(ctx_r, group, r) beforehand), each rank with its SRS slice, one thread per rank
static napi_value ProveGroup(napi_env env, napi_callback_info info) {
  size_t argc = 8;
  napi_value argv[8];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Job* j = new Job();
  j->op = 3;
  uint32_t W = 0;
  napi_get_array_length(env, argv[0], &W);
  for (uint32_t r = 0; r < W; r++) {
    napi_value e;
    napi_get_element(env, argv[0], r, &e);
    j->ranks.push_back(get_ctx(env, e));
  }
  size_t len = 0;
  napi_get_value_string_utf8(env, argv[1], nullptr, 0, &len);
  j->path.resize(len + 1);
  napi_get_value_string_utf8(env, argv[1], &j->path[0], len + 1, &len);
  j->path.resize(len);
  if (W < 1) {
    delete j;
    napi_throw_error(env, nullptr, "proveGroup: no ranks");
    return nullptr;
  }
  // the prove(...) argument list from `kind` on: argv[2..7] -> positions 1..6 (argv[0] unused)
  napi_value pa[8];
  pa[0] = argv[0];
  for (int i = 2; i < 8; i++) pa[i - 1] = argv[i];
  return prove_args(env, pa, argc - 1, j);
}

static napi_value prove_args(napi_env env, napi_value* argv, size_t argc, Job* j) {
  napi_get_value_int32(env, argv[1], &j->kind);
  napi_get_value_int32(env, argv[2], &j->nbits);
  uint32_t nf = 0, nt = 0;
  napi_get_array_length(env, argv[3], &nf);
  napi_get_array_length(env, argv[4], &nt);
  j->npols = (int)nf;
  for (uint32_t i = 0; i < nf; i++) {
    napi_value e;
    napi_get_element(env, argv[3], i, &e);
    j->f.push_back(view_of(env, e, j->refs));
    napi_get_element(env, argv[4], i, &e);
    j->t.push_back(view_of(env, e, j->refs));
  }
  napi_valuetype ty;
  napi_typeof(env, argv[5], &ty);
  if (ty != napi_null && ty != napi_undefined) {
    j->selected = true;
    j->sf = view_of(env, argv[5], j->refs);
    j->st = view_of(env, argv[6], j->refs);
  }
  if (argc > 7) {
    napi_typeof(env, argv[7], &ty);
    if (ty == napi_boolean) napi_get_value_bool(env, argv[7], &j->want_mont);
  }
  return queue(env, j, j->op == 3 ? "kgs_prove_group" : "kgs_prove");
}

// frOp(ctx, op, Uint8Array) -> Promise<Uint8Array> on ctx's GPU, elementwise over 32 B elements:
// op 0 = Fr.batchToMontgomery, 1 = Fr.batchFromMontgomery, 2 = Fr.batchInverse (0 -> 0),
// 3 = Fr.fft, 4 = Fr.ifft (2^k elements, natural order) — the curve shim's batch members
static napi_value FrOp(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Job* j = new Job();
  j->op = 2;
  j->ctx = get_ctx(env, argv[0]);
  napi_get_value_int32(env, argv[1], &j->fr_op);
  j->in = view_of(env, argv[2], j->refs);
  const uint64_t n = j->in.len / 32;
  const bool pow2 = n && !(n & (n - 1));
  const char* bad = j->fr_op < 0 || j->fr_op > 4                  ? "frOp: unknown op"
                    : !n || j->in.len % 32                        ? "frOp: the buffer must hold 32-byte elements"
                    : j->fr_op >= 3 && (!pow2 || n > (1ull << 28)) ? "frOp: fft size must be a power of two <= 2^28"
                                                                   : nullptr;
  if (bad) {
    for (napi_ref r : j->refs) napi_delete_reference(env, r);
    delete j;
    napi_throw_error(env, nullptr, bad);
    return nullptr;
  }
  return queue(env, j, "kgs_fr_op");
}

// verifyPtau(kind, ptauPath, nbits, npols, selected, commitments(Uint8Array), evaluations(Uint8Array))
// -> boolean (host-only pairing check, kgs_verify_ptau)
static napi_value VerifyPtau(napi_env env, napi_callback_info info) {
  size_t argc = 7;
  napi_value argv[7];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  int32_t kind = 0, nbits = 0, npols = 0;
  bool selected = false;
  napi_get_value_int32(env, argv[0], &kind);
  size_t plen = 0;
  napi_get_value_string_utf8(env, argv[1], nullptr, 0, &plen);
  std::string path(plen + 1, '\0');
  napi_get_value_string_utf8(env, argv[1], &path[0], plen + 1, &plen);
  path.resize(plen);
  napi_get_value_int32(env, argv[2], &nbits);
  napi_get_value_int32(env, argv[3], &npols);
  napi_get_value_bool(env, argv[4], &selected);
  std::vector<uint8_t> com = bytes_of(env, argv[5]), ev = bytes_of(env, argv[6]);
  int nc = 0, ne = 0;
  kgs_proof_shape(kind, npols, selected ? 1 : 0, &nc, &ne);
  if (com.size() != (size_t)nc * 64 || ev.size() != (size_t)ne * 32) {
    napi_throw_error(env, nullptr, "proof buffers do not match the proof shape");
    return nullptr;
  }
  int rc = kgs_verify_ptau(kind, path.c_str(), nbits, npols, selected ? 1 : 0, com.data(), ev.data());
  if (rc < 0) {
    napi_throw_error(env, nullptr, "kgs_verify_ptau failed");
    return nullptr;
  }
  napi_value out;
  napi_get_boolean(env, rc == 1, &out);
  return out;
}

// groupCreateLocal(world) -> rank group of `world` contexts in this process (kgs_group_create_local):
// the distributed prover with every vector sharded, driven from one Node process (one libuv
// thread per rank). ctxSetGroup(ctx, group|null, rank) attaches / detaches a context.
static void group_finalize(napi_env, void* data, void*) { kgs_group_destroy((kgs_group_t*)data); }
static napi_value GroupCreateLocal(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  int32_t world = 1;
  if (argc > 0) napi_get_value_int32(env, argv[0], &world);
  kgs_group_t* g = nullptr;
  if (kgs_group_create_local(world, &g) != KGS_OK) {
    napi_throw_error(env, nullptr, kgs_last_error());
    return nullptr;
  }
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, g, group_finalize, nullptr, &ext));
  return ext;
}
static napi_value CtxSetGroup(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  kgs_ctx_t* ctx = get_ctx(env, argv[0]);
  napi_valuetype ty;
  napi_typeof(env, argv[1], &ty);
  void* g = nullptr;
  if (ty == napi_external) napi_get_value_external(env, argv[1], &g);
  int32_t rank = 0;
  if (argc > 2) napi_get_value_int32(env, argv[2], &rank);
  if (kgs_ctx_set_group(ctx, (kgs_group_t*)g, rank) != KGS_OK) {
    napi_throw_error(env, nullptr, kgs_last_error());
    return nullptr;
  }
  return nullptr;
}

// ctxSetMsmLanes(ctx, lanes): 2 = the single-proof latency mode, 1 = throughput (several proofs in
// flight on the device) — kgs_ctx_set_msm_lanes; call while the context is idle
static napi_value CtxSetMsmLanes(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  kgs_ctx_t* ctx = get_ctx(env, argv[0]);
  int32_t lanes = 2;
  napi_get_value_int32(env, argv[1], &lanes);
  if (kgs_ctx_set_msm_lanes(ctx, lanes) != KGS_OK) {
    napi_throw_error(env, nullptr, kgs_last_error());
    return nullptr;
  }
  return nullptr;
}

// pairingEq(g1s, g2s): g1s = n x 64 B affine LEM G1, g2s = n x 128 B affine LEM G2 -> bool
// (curve.pairingEq, src/grandsum/mset_eq_kzg_verifier.js:182)
static napi_value PairingEq(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  std::vector<uint8_t> a = bytes_of(env, argv[0]), b = bytes_of(env, argv[1]);
  if (a.size() % 64 || b.size() % 128 || a.size() / 64 != b.size() / 128) {
    napi_throw_error(env, nullptr, "pairingEq: expected n x 64 B G1 and n x 128 B G2 affine points");
    return nullptr;
  }
  const int rc = kgs_pairing_eq((int)(a.size() / 64), a.data(), b.data());
  if (rc < 0) {
    napi_throw_error(env, nullptr, "pairingEq: point not on the curve");
    return nullptr;
  }
  napi_value out;
  napi_get_boolean(env, rc == 1, &out);
  return out;
}

// msmPoints(ctx, bases, scalarsStd) -> Promise<64 B affine LEM sum_i s_i P_i> on the GPU of ctx (the
// curve shim's G1.multiExpAffine, polynomial.js:1112, whose scalars are standard-form LE after
// Fr.batchFromMontgomery): the bases become ctx's resident point set. Async work like every other
// heavy call: the window-table build of the bases must not block the event loop.
static napi_value MsmPoints(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Job* j = new Job();
  j->op = 4;
  j->ctx = get_ctx(env, argv[0]);
  j->bases = bytes_of(env, argv[1]);
  j->scal = bytes_of(env, argv[2]);
  const uint64_t n = j->scal.size() / 32;
  if (j->scal.size() % 32 || j->bases.size() != 64 * n || n < 2) {
    delete j;
    napi_throw_error(env, nullptr, "msmPoints: expected n >= 2 affine LEM bases and n 32 B scalars");
    return nullptr;
  }
  return queue(env, j, "kgs_msm_points");
}

// lastTiming(ctx) -> [round 1..5 ms, -, input copy, prover, write-back wait] of the context's last
// kgs_prove call (kgs_last_timing; diagnostics, call when the context is idle)
static napi_value LastTiming(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  kgs_ctx_t* ctx = get_ctx(env, argv[0]);
  double t[9] = {0};
  const int n = kgs_last_timing(ctx, t, 9);
  napi_value arr;
  napi_create_array(env, &arr);
  for (int i = 0; i < n; i++) {
    napi_value v;
    napi_create_double(env, t[i], &v);
    napi_set_element(env, arr, (uint32_t)i, v);
  }
  return arr;
}

static napi_value Init(napi_env env, napi_value exports) {
  napi_property_descriptor desc[] = {
      {"ctxCreate", nullptr, CtxCreate, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"srsLoadPtau", nullptr, SrsLoad, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"srsInfo", nullptr, SrsInfo, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"prove", nullptr, Prove, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"keccak256", nullptr, Keccak, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"verifyPtau", nullptr, VerifyPtau, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"deviceCount", nullptr, DeviceCount, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"ptauPower", nullptr, PtauPower, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"pairingEq", nullptr, PairingEq, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"groupCreateLocal", nullptr, GroupCreateLocal, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"ctxSetGroup", nullptr, CtxSetGroup, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"msmPoints", nullptr, MsmPoints, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"proveGroup", nullptr, ProveGroup, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"lastTiming", nullptr, LastTiming, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"ctxSetMsmLanes", nullptr, CtxSetMsmLanes, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"frOp", nullptr, FrOp, nullptr, nullptr, nullptr, napi_default, nullptr},
  };
  napi_define_properties(env, exports, sizeof(desc) / sizeof(desc[0]), desc);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
