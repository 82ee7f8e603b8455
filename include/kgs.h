/* kgs.h — C-ABI of the MI355X-native KZG grand-sum / grand-product prover (libkgs.so).
 *
 * Drop-in boundary for the reference's hot path (xavi-pinsach/kzg-grandsums-study, JavaScript):
 * the reference has no native layer of its own; its arithmetic runs in the third-party
 * ffjavascript@0.2.59 / wasmcurves@0.2.1 wasm. Each entry point below names the reference
 * interface it replaces. Host bindings (N-API addon for the JS modules, ctypes for Python) are
 * shown in INTEGRATION.md.
 *
 * Conventions
 *  - Fr / Fq elements: 32 bytes little-endian. "mont" = Montgomery form with R = 2^256 (the
 *    in-memory form of every ffjavascript field element); "std" = standard form.
 *  - G1 affine points: 64 bytes x||y, each 32 B LE Montgomery Fq ("LEM", as in .ptau files and in
 *    ffjavascript `G1.toAffine` output); the point at infinity is 64 zero bytes.
 *  - Every call returns 0 on success or a negative KGS_E_* code; kgs_last_error() returns the
 *    message of the last failure on the calling thread. Semantic failures reproduce the
 *    reference's Error messages verbatim.
 *  - A context owns one HIP device, its HIP streams and work buffers. Every entry point taking a
 *    context holds that context's mutex for the whole call: calls on one context from several
 *    threads are serialised (a busy context blocks, it is never entered twice); independent
 *    contexts run concurrently. The SRS window tables and the NTT domain tables are read-only and
 *    shared by all contexts of a device (one copy per device, refcounted).
 */
#ifndef KGS_H
#define KGS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KGS_OK 0
#define KGS_E_ARG (-1)             /* bad argument / shape */
#define KGS_E_HIP (-2)             /* HIP runtime failure */
#define KGS_E_NOT_WELL_CALC (-3)   /* "The grand-sum polynomial S is not well calculated" (grandsum.js:56)
                                      "The grand-product polynomial Z is not well calculated" (grandproduct.js:51) */
#define KGS_E_NOT_DIVISIBLE (-4)   /* "Polynomial is not divisible" (polynomial.js:878) */
#define KGS_E_DOES_NOT_DIVIDE (-5) /* "Polynomial does not divide" (polynomial.js:847) */
#define KGS_E_IO (-6)              /* ptau read/write failure (binfileutils / ptau_utils.js:3-24) */
#define KGS_E_SRS (-7)             /* "The Powers of Tau file is not sufficiently large ..." (prover.js:79-81) */
#define KGS_E_COMM (-8)            /* the shard all-gather callback reported a failure */
#define KGS_E_RANGE (-9)           /* reference-quirks mode only: "offset is out of bounds", the V8 RangeError the
                                      reference's divZh throws for a zero quotient (polynomial.js:857,884) */

#define KGS_GRANDSUM 0
#define KGS_GRANDPRODUCT 1
/* Lookup (the commented-out cases of test/lookup_kzg_grandsum.test.js:24-44):
 * the selected grand-sum with sel_t carrying MULTIPLICITIES, so that
 *   sum_i selF_i / (f_i + gamma) == sum_i m_i / (t_i + gamma)
 * (f's selected values all occur in t). Identical to KGS_GRANDSUM with selectors in every respect
 * (transcript, proof layout, builder, error strings) except that the quotient and r(X) drop the
 * binary constraint on sel_t (the alpha^3 (selT - selT^2) term of prover.js:241-244 and
 * verifier.js:80-81). sel_f stays binary. Needs both selectors. Not in the reference, so parity is
 * against the oracle's restatement only. */
#define KGS_LOOKUP 2

typedef struct kgs_ctx kgs_ctx_t;

const char* kgs_last_error(void);
const char* kgs_version(void);

/* Number of visible HIP devices (the JS backend spreads its context pool over them). */
int kgs_device_count(int* count);
/* Create / destroy a context on HIP device `device`. kgs_ctx_destroy waits for a call still
 * running on the context. */
int kgs_ctx_create(int device, kgs_ctx_t** out);
void kgs_ctx_destroy(kgs_ctx_t* ctx);

/* ---- multi-GPU: MSM point-range sharding (replaces the [ffjs] worker-pool split
 * of G1.multiExpAffine, polynomial.js:1106-1115, by a split over one process per GPU).
 * With world > 1 every rank runs the whole prover on identical inputs; each commitment MSM over N
 * points is cut into `world` contiguous point ranges (kgs_shard_range), rank r runs Pippenger on
 * its range against the same resident SRS tables and the per-rank partials (c bit-sum points
 * T_k, XYZZ, 128 B each) are exchanged through `fn`, once per prover round. Every rank then
 * holds the same proof. `fn(user, send, recv, bytes)` must all-gather `bytes` from every rank
 * into recv (rank-major, world * bytes) and return 0; it is called in the same order on every
 * rank (the Python binding implements it over torch.distributed, i.e. RCCL on MI355X).
 * world == 1 turns sharding off. */
typedef int (*kgs_allgather_fn)(void* user, const uint8_t* send, uint8_t* recv, uint64_t bytes);
int kgs_ctx_set_shard(kgs_ctx_t* ctx, int rank, int world, kgs_allgather_fn fn, void* user);
/* rank's point range [lo, hi) of an n-point MSM: lo = floor(n*rank/world) */
int kgs_shard_range(uint64_t n, int rank, int world, uint64_t* lo, uint64_t* hi);
/* host-only: commitment from `nparts` rank partials (each c XYZZ points T_0..T_{c-1}, 128 B:
 * X,Y,ZZ,ZZZ LE Montgomery Fq, ZZ == 0 is infinity): sum_k 2^k sum_r T_k^(r) -> affine LEM */
int kgs_msm_combine(const uint8_t* T_all, int nparts, int c, uint8_t out_lem[64]);

/* ---- multi-GPU: the distributed prover (north_star: "the MSM and NTT
 * shard ... by scalar/point range and by butterfly stage across the 8 GPUs of one node").
 * A context attached to a group of W ranks (W = 1, 2, 4, 8 or 16; one context per rank) proves with
 * EVERY vector sharded: NTTs as a local transform + one all-to-all (CYCLIC <-> E layouts), the
 * grand-sum/product builder as a local scan + one all-gather of rank totals, the quotient and the
 * divisibility check on local slices with halo elements, Horner on CYCLIC slices, the synthetic
 * divisions on BLOCK slices with one all-gather of carries, and every MSM over the rank's slice of
 * the SRS. Each rank passes the FULL inputs (as for kgs_prove / kgs_prove_device) and receives the
 * identical, full proof (byte-identical to the single-GPU prover). Needs n >= 2 W^2.
 * All ranks must call the prover with the same arguments, in the same order. Each rank may hold the
 * whole SRS (kgs_srs_load_ptau: the MSMs read it with a point stride) or only its slice
 * (kgs_srs_load_ptau_slice(ctx, path, nbits, rank, world): 1/world of the tables).
 * Transports:
 *   local : several contexts of ONE process (one host thread per rank; devices may differ: attaching a
 *           context, kgs_ctx_set_group, enables peer access between its device and every other attached
 *           rank's device, and fails with KGS_E_COMM for a pair without peer access — the all-to-all
 *           then copies device to device over xGMI; UNVERIFIED on more than one device: every run of
 *           this build had one GPU, so all ranks shared a device)
 *   host  : any host all-gather callback (e.g. torch.distributed gloo); device data via the host
 *   rccl  : one process per GPU, RCCL over xGMI (rank 0 makes the id, the caller broadcasts it)
 * Failures:
 *   - rank-local preconditions (no / too small / wrong-slice SRS, pinned staging) are decided by all
 *     ranks together before the first exchange: every rank fails with the lowest failing rank's
 *     error and the group stays usable;
 *   - semantic prover errors (not well calculated / not divisible / does not divide) are decided
 *     from exchanged values, identically on every rank: the group stays usable;
 *   - anything else (HIP, allocation, transport) aborts the group: local / host peers fail at their
 *     next exchange; RCCL peers fail when their wait for the exchange passes the deadline
 *     KGS_GROUP_TIMEOUT_S (default 120 s; ncclCommAbort alone does not release them). The group is
 *     spent. The RCCL transport has run end to end with a one-rank communicator only (no multi-GPU
 *     box was available to this build); local-group runs of up to 16 ranks cover the data path. */
typedef struct kgs_group kgs_group_t;
int kgs_group_create_local(int world, kgs_group_t** out);
int kgs_group_create_host(int world, kgs_allgather_fn fn, void* user, kgs_group_t** out);
/* host transport with a real all-to-all: `a2a(user, send, recv, chunk)` sends chunk j of send (world
 * chunks of `chunk` bytes) to rank j and receives rank j's chunk for this rank into chunk j of recv
 * (e.g. torch.distributed all_to_all_single over gloo); returns 0. (W - 1) / W of a vector leaves a
 * rank per all-to-all, against W x the vector received through the all-gather-only transport. */
typedef int (*kgs_alltoall_fn)(void* user, const uint8_t* send, uint8_t* recv, uint64_t chunk);
int kgs_group_create_host_a2a(int world, kgs_allgather_fn fn, kgs_alltoall_fn a2a, void* user, kgs_group_t** out);
int kgs_group_rccl_unique_id(uint8_t id[128]);
int kgs_group_create_rccl(int rank, int world, const uint8_t id[128], int device, kgs_group_t** out);
void kgs_group_destroy(kgs_group_t* g);
int kgs_group_world(kgs_group_t* g, int* world);
/* attach (g != NULL) or detach (g == NULL) the distributed prover for this rank; a world-1 group
 * runs the distributed code path on one rank (exercises a transport end to end on one GPU) */
int kgs_ctx_set_group(kgs_ctx_t* ctx, kgs_group_t* g, int rank);
/* exchanges of the context's last proof (zeros after a single-GPU proof): out[0..5] = all-to-all
 * count, their summed span in ms (HIP events on the prover's stream around each exchange: the
 * transfer plus any wait for the peers), bytes that left this rank in them; host all-gather count,
 * their summed wall ms, bytes sent (bytes x (world - 1)). Returns the number of values written. */
int kgs_last_exchange(kgs_ctx_t* ctx, double* out, int max);

/* MSM lanes per context (default 2): with 2, the independent commitments of one prover round
 * (round 1's F_i / T_i, round 5's W_xi / W_xiw) alternate between two HIP streams with separate
 * work buffers, so one MSM's latency-bound tail overlaps the other's bucket accumulation
 * (single-proof latency -3 %, selected-vector 2^22 k=4 -7 %). Use 1 when several contexts already
 * keep the GPU busy with independent proofs (throughput). */
int kgs_ctx_set_msm_lanes(kgs_ctx_t* ctx, int lanes);

/* Reference-quirks mode (default ON since round 5: a new context is on unless the environment variable
 * KGS_REFERENCE_QUIRKS is "0"). On, the prover reproduces what the reference does on the degenerate
 * inputs where the reference does not compute the mathematical quotient (DESIGN.md §4 "Reference
 * quirks"); off (exact-math mode), it returns a valid proof for every valid
 * multiset. Detecting the degenerate inputs costs nothing measurable (93.0 proofs/s either way at
 * n = 2^20, profiles/r05/quirks_cost_ab.txt):
 *   - an operand of degree 1 <= d < n/2 (F, T, S/Z, selF, selT — e.g. F[i] = w^i): the reference's
 *     Polynomial.multiply evaluates it on the wrong points (polynomial.js:352-376 vs
 *     evaluations.js:12-18); the reference's quotient chain is then replayed on the GPU with the
 *     reference's buffer sizes and buffer sharing, and the prover fails where the reference fails
 *     ("Polynomial is not divisible", "Polynomial does not divide") or returns the proof it returns;
 *   - a zero quotient (e.g. F == T element by element): KGS_E_RANGE "offset is out of bounds".
 * Only the two reference arguments are affected (KGS_LOOKUP has no reference behaviour to follow). A
 * rank group (kgs_ctx_set_group) decides the degenerate cases from all-gathered degrees and replays
 * the chain on the gathered operands on every rank: every rank fails with the reference's error, or
 * returns the reference's proof. The replay reproduces transforms of up to 2^26 points (the
 * reference's own need n^2 points for a degree-1 operand); beyond that it fails with KGS_E_ARG.
 * One gap remains in rank groups: a replay that writes into polF's buffer (the unselected grand-sum's
 * polQ1.add(polF) on a shorter polQ1) makes a group fail with KGS_E_ARG where the
 * single-GPU prover follows the reference. No valid multiset of the test families reaches it with a
 * proof: the oracle restatement hits that write only on zero quotients (F == T), where the replay
 * first throws the reference's RangeError (DESIGN.md §13 "Q2 in rank groups"). */
int kgs_ctx_set_reference_quirks(kgs_ctx_t* ctx, int on);

/* Load a .ptau file (binfileutils layout, sections 1-3) and make the first 2^(nbits_max+1) G1
 * points device-resident, together with the MSM window tables and the NTT tables for domains
 * up to 2^nbits_max (nbits_max < 0: the file's power). Replaces readBinFile + readPTauHeader +
 * fd.readToBuffer(section 2) (src/grandsum/mset_eq_kzg_prover.js:15-16,83-85; src/ptau_utils.js:3-24),
 * which reads exactly domainSize*2 points per call: pass the proof's nBits as nbits_max.
 * Device SRS cache, grow-only: a context that already holds tables of the same file (same resolved
 * path, size and mtime) for a domain >= 2^nbits_max keeps them (no-op); tables of that file built
 * for a large enough domain by another context on the device are shared, not rebuilt. */
int kgs_srs_load_ptau(kgs_ctx_t* ctx, const char* path, int nbits_max);
/* A rank's slice of the SRS for the distributed prover (kgs_ctx_set_group, SURVEY.md §8e: "each GPU
 * holds only its SRS slice"): of the first 2^(nbits_max+1) points only rank + world * j are read,
 * made resident and window-expanded — 1/world of the tables of kgs_srs_load_ptau. Every MSM of the
 * distributed prover runs over the rank's CYCLIC slice, whose scalar j multiplies exactly point
 * rank + world * j, so this is all a rank needs. A context holding a slice proves only as that rank
 * of a group of that world (kgs_prove on it alone fails with KGS_E_ARG). Same grow-only cache. */
int kgs_srs_load_ptau_slice(kgs_ctx_t* ctx, const char* path, int nbits_max, int rank, int world);
/* slice of the resident SRS (world 1: the whole prefix) and the bytes of its window tables */
int kgs_srs_slice_info(kgs_ctx_t* ctx, int* rank, int* world, uint64_t* table_bytes);
/* Power of a ptau file from its header only (readPTauHeader, src/ptau_utils.js:3-24). */
int kgs_ptau_power(const char* path, int* power);
/* Same from in-memory LEM points (npts >= 2). `power` is the ceremony power to report. */
int kgs_srs_load_points(kgs_ctx_t* ctx, const uint8_t* g1_lem, uint64_t npts, int power, int nbits_max);
/* power of the loaded ptau, number of resident points, MSM window c */
int kgs_srs_info(kgs_ctx_t* ctx, int* power, uint64_t* npts, int* window_c);
/* Read [tau]_2 (128 B LEM, section 3 offset 128) from a ptau (verifier input,
 * src/grandsum/mset_eq_kzg_verifier.js:18-19). */
int kgs_ptau_read_tau_g2(const char* path, uint8_t out128[128]);

/* Write a synthetic ptau (sections 1-3 with the hermez layout; section 3 holds [1]_2 and
 * [tau]_2 only) for a known tau (32 B LE standard form). G1 powers are generated on the GPU of
 * `ctx` (or on the CPU if ctx == NULL). */
int kgs_ptau_write_synthetic(kgs_ctx_t* ctx, const char* path, int power, const uint8_t tau_std[32]);

/* Full prover — replaces mset_eq_kzg_{grandsum,grandproduct}_prover
 * (src/grandsum/mset_eq_kzg_prover.js:12, src/grandproduct/mset_eq_kzg_prover.js:12).
 *   kind      KGS_GRANDSUM | KGS_GRANDPRODUCT | KGS_LOOKUP (grand-sum layout; selectors required)
 *   nbits     domain size n = 2^nbits (1 <= nbits <= SRS nbits_max)
 *   npols     k >= 1 (vector argument when k > 1)
 *   evals_f/t k host pointers, n x 32 B STANDARD-form evaluations each (the caller's
 *             Evaluations.eval before prover.js:147-148)
 *   sel_f/t   n x 32 B MONTGOMERY selector evaluations, or both NULL (unselected; the wrapper
 *             passes NULL when both are all Fr.one, prover.js:63-68)
 *   mont_f/t  optional k output pointers (n x 32 B) receiving the Montgomery evaluations that the
 *             reference writes back into the caller's objects (prover.js:147-148); may be NULL
 *   commitments_out  (#commitments x 64 B LEM), order:
 *             grand-sum:     F0,T0,..,F{k-1},T{k-1}, [selF,selT], S, Q, Wxi, Wxiw
 *             grand-product: F0,T0,..,F{k-1},T{k-1}, [selF,selT], Z, Q, Wxi, Wxiw
 *   evaluations_out  (#evaluations x 32 B Montgomery), order:
 *             grand-sum:     f0,t0,..,f{k-1},t{k-1}, [selF,selT], sxiw
 *             grand-product: f0,..,f{k-1}, [selF,selT], zxiw
 */
int kgs_prove(kgs_ctx_t* ctx, int kind, int nbits, int npols, const uint8_t* const* evals_f,
              const uint8_t* const* evals_t, const uint8_t* sel_f, const uint8_t* sel_t, uint8_t* const* mont_f,
              uint8_t* const* mont_t, uint8_t* commitments_out, uint8_t* evaluations_out);
/* Host-buffer boundary: kgs_prove copies pageable inputs into pinned staging (pieces overlapped with
 * their DMA) and the Montgomery outputs back out of it. Buffers the caller has pinned — hipHostMalloc
 * or kgs_host_register, for buffers reused across proofs — are DMA'd in place with no staging copy;
 * kgs_host_unregister before freeing a registered buffer. Registration costs more than one copy
 * (profiles/r03/boundary_ab.txt): register only buffers that outlive several proofs. */
int kgs_host_register(void* ptr, uint64_t bytes);
int kgs_host_unregister(void* ptr);
/* Every kgs_prove / kgs_prove_device call returns with none of its transfers or kernels pending, on
 * its error paths too (a failed call drains the context's streams before it returns), so a caller may
 * unregister or free its buffers as soon as the call returns. kgs_ctx_idle reports 1 when no stream
 * of the context has work outstanding, 0 otherwise (diagnostic; the tests check the contract). */
int kgs_ctx_idle(kgs_ctx_t* ctx);
/* Same with device-resident inputs (HIP device pointers on ctx's device). */
int kgs_prove_device(kgs_ctx_t* ctx, int kind, int nbits, int npols, const void* const* d_evals_f,
                     const void* const* d_evals_t, const void* d_sel_f, const void* d_sel_t, uint8_t* commitments_out,
                     uint8_t* evaluations_out);
/* number of commitments / evaluations a proof of this shape produces */
int kgs_proof_shape(int kind, int npols, int selected, int* n_commitments, int* n_evaluations);

/* ---- verifiers (host only; no context, no GPU) -------------------------------------------
 * mset_eq_kzg_grandsum_verifier / mset_eq_kzg_grandproduct_verifier
 * (src/grandsum/mset_eq_kzg_verifier.js:9, src/grandproduct/mset_eq_kzg_verifier.js:9): commitment
 * and evaluation buffers in the fixed order kgs_prove writes (kgs_proof_shape; KGS_LOOKUP proofs
 * are checked with kind KGS_LOOKUP and selected = 1); tau_g2 = [tau]_2 as
 * 128 B LEM (the second point of ptau section 3, kgs_ptau_read_tau_g2). Returns 1 (valid), 0
 * (invalid: not on G1, evaluation >= r, or the pairing equation fails) or a negative error. */
int kgs_verify(int kind, int nbits, int npols, int selected, const uint8_t* commitments, const uint8_t* evaluations,
               const uint8_t tau_g2[128]);
int kgs_verify_ptau(int kind, const char* ptau_path, int nbits, int npols, int selected, const uint8_t* commitments,
                    const uint8_t* evaluations);
/* curve.pairingEq (src/grandsum/mset_eq_kzg_verifier.js:182, src/grandproduct/mset_eq_kzg_verifier.js:177;
 * [ffjs] bn128 optimal-ate pairing): 1 if prod_k e(P_k, Q_k) == 1, 0 if not. P_k: affine LEM G1
 * (64 B, Montgomery; (0, 0) = infinity), Q_k: affine LEM G2 (128 B: x.c0, x.c1, y.c0, y.c1). Points
 * off their curve: KGS_E_ARG. Host only. */
int kgs_pairing_eq(int npairs, const uint8_t* g1_lem, const uint8_t* g2_lem);

/* Per-proof timing of the last kgs_prove* call (milliseconds, host wall clock): [0..4] prover rounds
 * 1-5, [5] unused, and for kgs_prove (host buffers) [6] input copy into pinned staging, [7] the
 * prover, [8] wait for the Montgomery write-back to the caller. Returns the number written. */
int kgs_last_timing(kgs_ctx_t* ctx, double* rounds_ms, int max_rounds);

/* ---- primitives (host buffers in/out; used by tests and by the bench's roofline legs) ---- */
/* [ffjs] Fr.batchToMontgomery */
int kgs_fr_to_mont(kgs_ctx_t* ctx, const uint8_t* in_std, uint8_t* out_mont, uint64_t n);
/* [ffjs] Fr.batchFromMontgomery (polynomial.js:1112): out = in * 2^-256, canonical */
int kgs_fr_from_mont(kgs_ctx_t* ctx, const uint8_t* in_mont, uint8_t* out_std, uint64_t n);
/* [ffjs] Fr.batchInverse (grandsum.js:41, grandproduct.js:36): out[i] = in[i]^-1, zero stays zero */
int kgs_fr_batch_inverse(kgs_ctx_t* ctx, const uint8_t* in_mont, uint8_t* out_mont, uint64_t n);
/* [ffjs] Fr.fft / Fr.ifft: natural order in and out, size 2^logm, ifft includes 1/m */
int kgs_ntt(kgs_ctx_t* ctx, const uint8_t* in_mont, uint8_t* out_mont, int logm, int inverse);
/* [ffjs] G1.multiExpAffine(SRS[0..n), fromMont(scalars)) + toAffine (polynomial.js:1106-1115) */
int kgs_msm(kgs_ctx_t* ctx, const uint8_t* scalars_mont, uint64_t n, uint8_t out_lem[64]);
/* ComputeSGrandSumPolynomial / ComputeZGrandProductPolynomial evaluations before the ifft
 * (grandsum.js:6-57, grandproduct.js:6-52): out = S (or Z) evaluations, natural order */
int kgs_grand_build(kgs_ctx_t* ctx, int kind, const uint8_t* f_mont, const uint8_t* t_mont, const uint8_t* sel_f,
                    const uint8_t* sel_t, const uint8_t gamma_mont[32], uint64_t n, uint8_t* out_mont);
/* Polynomial.evaluate (polynomial.js:228-238) */
int kgs_poly_eval(kgs_ctx_t* ctx, const uint8_t* coef_mont, uint64_t len, const uint8_t x_mont[32],
                  uint8_t out_mont[32]);
/* Polynomial.divByXSubValue (polynomial.js:814-851); out has `len` coefficients */
int kgs_poly_div_x_sub(kgs_ctx_t* ctx, const uint8_t* coef_mont, uint64_t len, const uint8_t z_mont[32],
                       uint8_t* out_mont);
/* Keccak-256 (js-sha3 keccak256) */
int kgs_keccak256(const uint8_t* data, uint64_t len, uint8_t out[32]);

/* ---- device timing helpers for bench.py (events recorded on ctx's stream) ---- */
/* Run `reps` MSMs of n scalars (device pointer) back to back; returns total ms on the stream. */
int kgs_bench_msm(kgs_ctx_t* ctx, const void* d_scalars_mont, uint64_t n, int reps, double* ms);
/* Run `reps` MSMs of n scalars, accumulating per-phase device time (ms) into phase_ms[4]:
 * [0] digit recoding + counting sort, [1] bucket accumulation (the k_accumulate launch alone),
 * [2] bucket combine, [3] bit-sum reduction. *entries = nonzero (bucket, point) entries of the last run. */
int kgs_bench_msm_phases(kgs_ctx_t* ctx, const void* d_scalars_mont, uint64_t n, int reps, double* phase_ms,
                         uint64_t* entries);
/* Run `reps` forward+inverse NTT pairs of size 2^logm on a device buffer; returns ms. */
int kgs_bench_ntt(kgs_ctx_t* ctx, void* d_buf, int logm, int reps, double* ms);
/* Host-only test hook of kgs_prove's staging copy (no GPU): copies len bytes src -> dst the way a
 * host input vector is staged (256 KiB pieces over the copy pool, spans of `span` bytes reported in
 * order once copied). spans_out[i] receives the byte offset of the i-th reported span (up to max);
 * fail_at >= 0 makes the report of span fail_at fail, the way a failed DMA enqueue does: the copy
 * then still completes and the call returns KGS_E_HIP. *nspans = spans reported. */
int kgs_test_stream_copy(uint8_t* dst, const uint8_t* src, uint64_t len, uint64_t span, int fail_at,
                         uint64_t* spans_out, int max, int* nspans);

#ifdef __cplusplus
}
#endif
#endif /* KGS_H */
