// BN254-G1 multi-scalar multiplication for gfx950 — replaces [ffjs] `G1.multiExpAffine` +
// `G1.toAffine` + `Fr.batchFromMontgomery` (polynomial.js:1106-1115).
//
// Design (MI355X-first):
//  * The SRS is fixed across proofs, so each base P_i is expanded ONCE into W = ceil(255/c)
//    window copies 2^(c*j)·P_i (affine, 64 B, table[j][i]; 1.7-2 GB at n = 2^20 — HBM is 288 GB).
//    A commitment then needs a single set of B = 2^(c-1) signed-digit buckets shared by all
//    windows: no per-window bucket reduction and no serial 2^c-doubling window combine.
//  * scalars leave Montgomery form and are recoded into W signed c-bit digits (digit kernel);
//  * counting sort of the N*W (digit -> point) entries by bucket (histogram, scan, scatter);
//  * bucket accumulation over FIXED-SIZE segments of the sorted array (load balanced whatever
//    the bucket sizes): one XYZZ mixed-add chain per segment, runs that straddle a segment
//    boundary are written as partials and merged by a per-bucket combine kernel;
//  * sum_b b·S_b = sum_k 2^k T_k with T_k = sum_{b has bit k} S_b: c independent tree
//    reductions (chip-parallel), then the c-term Horner + affine conversion on the host.
#include "kernels.hpp"
#include "field29.hpp"

namespace kgs {

static inline unsigned nb(uint64_t work, unsigned bs = 256) { return (unsigned)((work + bs - 1) / bs); }
constexpr int NH_MAX = MSM_NH_MAX;  // bucket-sort partitions (kernels.hpp msm_lob)

// ------------------------------------------------------------------ window table precompute
__global__ void __launch_bounds__(256) k_tab_dbl(uint32_t* __restrict__ tmp, const uint32_t* __restrict__ prev,
                                                 uint64_t npts, int c) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npts) return;
  g1_aff a = g1_aff::load(prev + 16 * i);
  g1_xyzz r = g1_xyzz::from_aff(a);
  for (int k = 0; k < c; k++) r = r.dbl();
  r.store(tmp + 32 * i);
}

// XYZZ -> affine with a per-thread Montgomery batch inversion over CH consecutive points.
template <int CH>
__global__ void __launch_bounds__(256) k_batch_affine(uint32_t* __restrict__ out, const uint32_t* __restrict__ in,
                                                      uint32_t* __restrict__ scratch, uint64_t npts) {
  KGS_AUX_PRIO();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t start = t * CH;
  if (start >= npts) return;
  const uint64_t end = start + CH < npts ? start + CH : npts;
  fq acc = fq::one();
  for (uint64_t i = start; i < end; i++) {
    acc.store(scratch + 8 * i);  // prefix product before i
    fq zz = fq::load(in + 32 * i + 16), zzz = fq::load(in + 32 * i + 24);
    if (!zz.is_zero()) acc = acc * (zz * zzz);
  }
  fq inv = acc.inverse();
  for (uint64_t i = end; i-- > start;) {
    fq zz = fq::load(in + 32 * i + 16), zzz = fq::load(in + 32 * i + 24);
    if (zz.is_zero()) {
      fq::zero().store(out + 16 * i);
      fq::zero().store(out + 16 * i + 8);
      continue;
    }
    fq pre = fq::load(scratch + 8 * i);
    fq zinv = inv * pre;  // 1/(ZZ*ZZZ)
    inv = inv * (zz * zzz);
    fq x = fq::load(in + 32 * i) * (zinv * zzz);
    fq y = fq::load(in + 32 * i + 8) * (zinv * zz);
    x.store(out + 16 * i);
    y.store(out + 16 * i + 8);
  }
}

// table coordinates x*2^256 -> x*2^261 (the fq29 Montgomery form of the bucket accumulation)
__global__ void __launch_bounds__(256) k_tab_to29(uint32_t* __restrict__ table, uint64_t nelem) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nelem) return;
  fq c;
#pragma unroll
  for (int k = 0; k < 8; k++) c.v[k] = f29::C261W[k];
  (fq::load(table + 8 * i) * c).store(table + 8 * i);
}

void msm_build_table(hipStream_t st, uint32_t* table, uint64_t npts, int c, int W, uint32_t* tmp_xyzz,
                     uint32_t* scratch) {
  for (int j = 1; j < W; j++) {
    const uint32_t* prev = table + (uint64_t)(j - 1) * npts * 16;
    uint32_t* cur = table + (uint64_t)j * npts * 16;
    hipLaunchKernelGGL(k_tab_dbl, dim3(nb(npts)), dim3(256), 0, st, tmp_xyzz, prev, npts, c);
    hipLaunchKernelGGL(k_batch_affine<32>, dim3(nb((npts + 31) / 32)), dim3(256), 0, st, cur, tmp_xyzz,
                       scratch, npts);
  }
  hipLaunchKernelGGL(k_tab_to29, dim3(nb(2 * (uint64_t)W * npts)), dim3(256), 0, st, table, 2 * (uint64_t)W * npts);
}

// ------------------------------------------------------------------ digits + two-pass bucket sort
// Entry (j, i) = (window, point) with signed digit d = digit_j(from_mont(scalar_i)); key |d| in
// [0, B], B = 2^(c-1); key 0 entries are dropped. Sort by key without global per-entry atomics:
//  sorting is by k' = key - 1 in [0, B) (c - 1 bits): pass 1 partitions by p = k' >> LOB
//          (NH = B >> LOB <= NH_MAX = 2048 partitions of 2^LOB <= 256 keys each; NH = 256 up to c = 17,
//          2^(c-9) above: c = 20 has 2048). Per-block partition counts come from a histogram pass whose
//          block x partition table is scanned; each block then counting-sorts its entries in LDS
//          and writes them out as contiguous per-partition runs (coalesced stores instead of one
//          scattered 4 B + 1 B store per entry). Digits are RECOMPUTED from the scalars in both
//          passes instead of being materialised (one Montgomery product per scalar);
//  pass 2 sorts every partition by lo = key - (p << LOB) inside one workgroup, tile by tile
//          through LDS (again run-wise stores), and writes the bucket offsets.
// Order inside a bucket is unspecified (point addition is commutative).
// digits of scalar i: from the Montgomery-form scalars (STD = false) or from their standard forms
// (STD = true: k_sort_hist stores them for k_sort_part, which then skips the conversion)
template <int C, bool STD = false>
__device__ __forceinline__ void scalar_digits(int32_t (&d)[(255 + C - 1) / C], const uint32_t* sc, uint64_t i,
                                              uint32_t* std_out = nullptr) {
  constexpr int W = (255 + C - 1) / C;
  fr s = STD ? fr::load(sc + 8 * i) : fr::load(sc + 8 * i).from_mont();
  if (std_out) s.store(std_out + 8 * i);
  constexpr int32_t half = 1 << (C - 1);
  constexpr uint32_t mask = (1u << C) - 1;
  uint32_t carry = 0;
#pragma unroll
  for (int j = 0; j < W; j++) {
    const int bit = j * C;
    const int limb = bit >> 5, off = bit & 31;
    uint64_t w = limb < 8 ? s.v[limb] : 0;
    if (limb + 1 < 8) w |= (uint64_t)s.v[limb + 1] << 32;
    int32_t v = (int32_t)((w >> off) & mask) + (int32_t)carry;
    carry = v > half ? 1u : 0u;
    d[j] = carry ? v - (1 << C) : v;
  }
}

// exclusive scan of a[0..n), n <= 256, by the 64 lanes of ONE wave (4 elements per lane); out may alias a
__device__ __forceinline__ uint32_t wave_excl_scan256(const uint32_t* a, uint32_t* out, int n) {
  const int lane = threadIdx.x & 63;
  uint32_t x[4], local = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int idx = lane * 4 + k;
    x[k] = idx < n ? a[idx] : 0;
    local += x[k];
  }
  uint32_t incl = local;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off);
    if (lane >= off) incl += y;
  }
  uint32_t run = incl - local;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int idx = lane * 4 + k;
    if (idx < n) out[idx] = run;
    run += x[k];
  }
  return __shfl(incl, 63);  // total
}

// exclusive scan of a[0..n) by all NT threads of the block (n <= NH_MAX: up to 8 elements per thread
// at NT = 256); tmp: NT words of LDS; out may alias a; ends with a barrier; returns the total
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(const uint32_t* a, uint32_t* out, int n, uint32_t* tmp) {
  const int t = threadIdx.x;
  const int per = (n + NT - 1) / NT;
  const int lo = t * per < n ? t * per : n, hi = lo + per < n ? lo + per : n;
  uint32_t sum = 0;
  for (int i = lo; i < hi; i++) sum += a[i];
  tmp[t] = sum;
  __syncthreads();
  for (int off = 1; off < NT; off <<= 1) {
    const uint32_t v = t >= off ? tmp[t - off] : 0u;
    __syncthreads();
    tmp[t] += v;
    __syncthreads();
  }
  uint32_t run = t ? tmp[t - 1] : 0u;
  const uint32_t total = tmp[NT - 1];
  for (int i = lo; i < hi; i++) {
    const uint32_t v = a[i];
    out[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

// partition of a nonzero digit magnitude: (key - 1) >> lob
__device__ __forceinline__ uint32_t part_of(uint32_t key, int lob) { return (key - 1) >> lob; }

#ifndef KGS_SORT_SPT
#define KGS_SORT_SPT 2
#endif
constexpr int SORT_SPT = KGS_SORT_SPT;  // scalars per thread in the histogram / partition passes

template <int C>
__global__ void __launch_bounds__(256) k_sort_hist(uint32_t* __restrict__ bh, const uint32_t* __restrict__ sc,
                                                   uint64_t N, int lob, int NH, uint32_t nblk,
                                                   uint32_t* __restrict__ std_out) {
  KGS_AUX_PRIO();
  // per-block partition histogram, stored transposed: bh[p * nblk + block]
  constexpr int W = (255 + C - 1) / C;
  __shared__ uint32_t h[NH_MAX];
  for (int t = threadIdx.x; t < NH; t += 256) h[t] = 0;
  __syncthreads();
  for (int q = 0; q < SORT_SPT; q++) {
    const uint64_t i = ((uint64_t)blockIdx.x * SORT_SPT + q) * 256 + threadIdx.x;
    if (i < N) {
      int32_t d[W];
      scalar_digits<C>(d, sc, i, std_out);
#pragma unroll
      for (int j = 0; j < W; j++) {
        if (d[j]) atomicAdd(&h[part_of((uint32_t)(d[j] < 0 ? -d[j] : d[j]), lob)], 1u);
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < NH; t += 256) bh[(uint64_t)t * nblk + blockIdx.x] = h[t];
}

// grid = NH workgroups: exclusive scan of one partition's per-block counts (in place) and its total
__global__ void __launch_bounds__(256) k_sort_scan_blocks(uint32_t* __restrict__ bh, uint32_t* __restrict__ ptot,
                                                          uint32_t nblk) {
  KGS_AUX_PRIO();
  __shared__ uint32_t part[256];
  uint32_t* row = bh + (uint64_t)blockIdx.x * nblk;
  const uint32_t per = (nblk + 255) / 256;
  const uint32_t lo = threadIdx.x * per, hi = lo + per < nblk ? lo + per : nblk;
  uint32_t s = 0;
  for (uint32_t b = lo; b < hi; b++) s += row[b];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (uint32_t b = lo; b < hi; b++) {
    uint32_t v = row[b];
    row[b] = run;
    run += v;
  }
  if (threadIdx.x == 255) ptot[blockIdx.x] = part[255];
}

__device__ __forceinline__ uint32_t chunk_count(uint32_t size);

// hi_off[p] = exclusive scan of partition totals (NH <= NH_MAX); offsets[B+1] = total; cpre = exclusive
// scan of the lo pass's chunks per partition (cpre[NH] = all chunks); bpart[b] = the partition of
// lo-pass block b (its chunk is b - cpre[bpart[b]])
__global__ void __launch_bounds__(256) k_sort_scan(uint32_t* __restrict__ hi_off, const uint32_t* __restrict__ ptot,
                                                   int NH, uint32_t* __restrict__ offsets, uint32_t B,
                                                   uint32_t* __restrict__ cpre, uint32_t* __restrict__ bpart) {
  KGS_AUX_PRIO();
  __shared__ uint32_t gp[NH_MAX], tmp[256];
  const uint32_t total = block_excl_scan<256>(ptot, hi_off, NH, tmp);
  for (int q = threadIdx.x; q < NH; q += 256) gp[q] = chunk_count(ptot[q]);
  __syncthreads();
  const uint32_t chunks = block_excl_scan<256>(gp, cpre, NH, tmp);
  for (int q = threadIdx.x; q < NH; q += 256) {
    const uint32_t b0 = cpre[q];
    for (uint32_t g = 0; g < gp[q]; g++) bpart[b0 + g] = (uint32_t)q;
  }
  if (threadIdx.x == 0) {
    hi_off[NH] = total;
    cpre[NH] = chunks;
    offsets[0] = 0;  // key 0 (zero digits) is never stored
    offsets[B + 1] = total;
  }
}

// dynamic LDS (part_lds in msm_run): NS = 256 * SORT_SPT * W staged entries (4 B value, 2 B partition,
// 1 B lo) and the block's per-partition base / offset / cursor (3 x NH words)
// scalar i multiplies SRS point pbase + pstride * i (a contiguous or strided slice of the SRS)
template <int C>
__global__ void __launch_bounds__(256) k_sort_part(uint32_t* __restrict__ tval, uint8_t* __restrict__ tlo,
                                                   const uint32_t* __restrict__ bh, const uint32_t* __restrict__ ptot,
                                                   const uint32_t* __restrict__ hi_off, const uint32_t* __restrict__ sc,
                                                   uint64_t N, uint64_t Nsrs, uint64_t pbase, uint64_t pstride, int lob,
                                                   int NH, uint32_t nblk) {
  KGS_AUX_PRIO();
  constexpr int W = (255 + C - 1) / C;
  extern __shared__ uint32_t smem[];
  constexpr int NS = 256 * SORT_SPT * W;
  uint32_t* sval = smem;                          // NS values
  uint32_t* base = smem + NS;                     // NH each
  uint32_t* loff = base + NH;
  uint32_t* cur = loff + NH;
  uint16_t* spart = (uint16_t*)(cur + NH);        // NS partitions (< NH_MAX)
  uint8_t* slo = (uint8_t*)(spart + NS);          // NS lo keys (< 2^LOB <= 256)
  __shared__ uint32_t tmp[256];
  const uint32_t blk = blockIdx.x, tid = threadIdx.x;
  for (int t = tid; t < NH; t += 256) {
    const uint32_t mine = bh[(uint64_t)t * nblk + blk];
    const uint32_t nxt = blk + 1 < nblk ? bh[(uint64_t)t * nblk + blk + 1] : ptot[t];
    base[t] = hi_off[t] + mine;
    cur[t] = nxt - mine;  // this block's count, scanned below
  }
  __syncthreads();
  const uint32_t tot = block_excl_scan<256>(cur, loff, NH, tmp);
  for (int t = tid; t < NH; t += 256) cur[t] = loff[t];
  __syncthreads();
  for (int q = 0; q < SORT_SPT; q++) {
    const uint64_t i = ((uint64_t)blk * SORT_SPT + q) * 256 + tid;
    if (i < N) {
      int32_t d[W];
      scalar_digits<C, true>(d, sc, i);  // sc: the standard forms k_sort_hist stored
      // entry values are 32-bit (point index | sign bit 31): the index arithmetic in 32 bits
      const uint32_t pidx = (uint32_t)pbase + (uint32_t)pstride * (uint32_t)i;
#pragma unroll
      for (int j = 0; j < W; j++) {
        if (!d[j]) continue;
        const uint32_t k = (uint32_t)(d[j] < 0 ? -d[j] : d[j]);
        const uint32_t p = part_of(k, lob);
        const uint32_t pos = atomicAdd(&cur[p], 1u);
        sval[pos] = ((uint32_t)j * (uint32_t)Nsrs + pidx) | (d[j] < 0 ? 0x80000000u : 0u);
        spart[pos] = (uint16_t)p;
        slo[pos] = (uint8_t)((k - 1) - (p << lob));
      }
    }
  }
  __syncthreads();
  for (uint32_t e = tid; e < tot; e += 256) {
    const uint32_t p = spart[e];
    const uint32_t g = base[p] + (e - loff[p]);
    tval[g] = sval[e];
    tlo[g] = slo[e];
  }
}

// Pass 2: every partition p is cut into G_p chunks; (1) per-chunk LDS histograms of lo, (2) every
// chunk's workgroup derives its per-lo global bases from its partition's chunk histograms (a 256-wide
// scan; the chunk-0 workgroup also writes the bucket offsets), counting-sorts its entries through LDS
// and writes each bucket's run with consecutive lanes.
// G_p = clamp(ceil(size_p / SL_CHUNK), 1, SL_G) and a chunk fits ONE LDS tile, so each bucket leaves
// a chunk as one run of ~SL_CHUNK / 256 entries: ~240 B at 2^20 points (2^20 / 256 partitions x 15
// windows = 61 K entries = 4 chunks of 15.4 K), write amplification ~1 + 32 B / run. 4 chunks per
// partition also make 1024 workgroups = exactly two rounds of 2 per CU at 2^20 (2048 = four at 2^21)
// where 12 K-entry chunks made 1280 (two and a half rounds).
// A/B knobs (-D): threads per k_lo_scatter block, entries per chunk (= LDS tile), max chunks per
// partition
#ifndef KGS_SL_THREADS
#define KGS_SL_THREADS 1024
#endif
#ifndef KGS_SL_CHUNK
#define KGS_SL_CHUNK 16384
#endif
#ifndef KGS_SL_G
#define KGS_SL_G 64
#endif
constexpr int SL_THREADS = KGS_SL_THREADS;
constexpr int SL_TILE = KGS_SL_CHUNK;
constexpr int SL_TILE_BIG = SL_TILE / 2;  // tiles of the multi-tile (skewed) path: 8 entries per thread
constexpr int SL_G = KGS_SL_G;
constexpr uint32_t SL_CHUNK = KGS_SL_CHUNK;
static_assert(SL_G <= MSM_SL_G_MAX, "lo-pass count buffer (prover.cpp msm_locnt)");
static_assert(SL_TILE % SL_THREADS == 0 && SL_TILE_BIG % SL_THREADS == 0, "lo-pass tile per thread");
// waves per SIMD the k_lo_scatter build targets (its VGPR budget): a 1024-thread block is 4 waves per
// SIMD, and at 8 it stays within 64 VGPRs
#ifndef KGS_SL_WPE
#define KGS_SL_WPE 8
#endif
constexpr int LC_THREADS = 256;  // k_lo_count: one wave per sub-histogram
constexpr int SL_HIST = LC_THREADS / 64;

// chunks of a partition of `size` entries
__device__ __forceinline__ uint32_t chunk_count(uint32_t size) {
  const uint32_t g = (size + SL_CHUNK - 1) / SL_CHUNK;
  return g < 1 ? 1u : g > (uint32_t)SL_G ? (uint32_t)SL_G : g;
}

// The lo-pass kernels run one workgroup per (partition, chunk) on a 1-D grid: cpre[p] = chunks of
// the partitions before p (k_sort_scan), block b belongs to the partition p = bpart[b] with
// cpre[p] <= b < cpre[p + 1]; blocks past cpre[NH] (the host sizes the grid by an upper bound) exit.
// (p, g, G) of block b and the partition's range [s0, s1) in two dependent rounds of loads (the table
// bpart replaces round 3's LDS copy of cpre / hi_off and its binary search, which at up to 2048
// partitions would take 16 KB of LDS per block). Uniform per block.
__device__ __forceinline__ bool chunk_of_block(const uint32_t* __restrict__ cpre, const uint32_t* __restrict__ hi_off,
                                               const uint32_t* __restrict__ bpart, int NH, uint32_t b, uint32_t& p,
                                               uint32_t& g, uint32_t& G, uint32_t& s0, uint32_t& s1) {
  const uint32_t nchunks = cpre[NH];
  if (b >= nchunks) return false;
  p = bpart[b];
  const uint32_t c0 = cpre[p], c1 = cpre[p + 1];
  g = b - c0;
  G = c1 - c0;
  s0 = hi_off[p];
  s1 = hi_off[p + 1];
  return true;
}

__device__ __forceinline__ void chunk_range(uint32_t s0, uint32_t s1, uint32_t G, uint32_t g, uint32_t& c0,
                                            uint32_t& c1) {
  const uint32_t csz = (s1 - s0 + G - 1) / G;
  c0 = s0 + g * csz < s1 ? s0 + g * csz : s1;
  c1 = c0 + csz < s1 ? c0 + csz : s1;
}

// one block per (partition, chunk): locnt[(p * nb + lo) * SL_G + g] = #entries of chunk g of
// partition p with this lo. 16-byte loads of the lo bytes (four in flight per thread), one
// sub-histogram per wave against LDS atomic contention.
__global__ void __launch_bounds__(LC_THREADS) k_lo_count(uint32_t* __restrict__ locnt, const uint8_t* __restrict__ tlo,
                                                         const uint32_t* __restrict__ hi_off,
                                                         const uint32_t* __restrict__ cpre,
                                                         const uint32_t* __restrict__ bpart, int NH, int lob) {
  KGS_AUX_PRIO();
  __shared__ uint32_t cnt[SL_HIST][256];
  uint32_t p, g, G, s0, s1;
  if (!chunk_of_block(cpre, hi_off, bpart, NH, blockIdx.x, p, g, G, s0, s1)) return;  // uniform per block
  const int nb = 1 << lob;
  const uint32_t tid = threadIdx.x;
  uint32_t c0, c1;
  chunk_range(s0, s1, G, g, c0, c1);
  for (uint32_t i = tid; i < SL_HIST * 256; i += LC_THREADS) (&cnt[0][0])[i] = 0;
  __syncthreads();
  uint32_t* h = cnt[tid >> 6];
  const uint32_t a0 = ((c0 + 15) & ~15u) < c1 ? (c0 + 15) & ~15u : c1;
  const uint32_t a1 = (c1 & ~15u) > a0 ? c1 & ~15u : a0;
  if (c0 + tid < a0) atomicAdd(&h[tlo[c0 + tid]], 1u);  // head: < 16 bytes
  if (a1 + tid < c1) atomicAdd(&h[tlo[a1 + tid]], 1u);  // tail: < 16 bytes
  const uint4* q4 = reinterpret_cast<const uint4*>(tlo);
  uint32_t q = a0 / 16 + tid;
  for (; q + 3 * LC_THREADS < a1 / 16; q += 4 * LC_THREADS) {  // four 16-byte loads in flight
    uint4 x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = q4[q + u * LC_THREADS];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t w[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
      for (int k = 0; k < 16; k++) atomicAdd(&h[(w[k >> 2] >> (8 * (k & 3))) & 255u], 1u);
    }
  }
  for (; q < a1 / 16; q += LC_THREADS) {
    const uint4 x = q4[q];
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 16; k++) atomicAdd(&h[(w[k >> 2] >> (8 * (k & 3))) & 255u], 1u);
  }
  __syncthreads();
  if ((int)tid < nb) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < SL_HIST; k++) v += cnt[k][tid];
    locnt[((uint64_t)p * nb + tid) * SL_G + g] = v;
  }
}

// write the runs of a sorted LDS tile: bucket b's run sv[src[b], + n[b]) -> sorted[dst[b], ...). A
// run of up to SL_BIGRUN entries is stored by one wave with consecutive lanes (uniform scalars: ~60
// entries per bucket per chunk); longer runs (skewed scalars: one bucket holds the whole chunk) by
// the whole block, so no wave is left with the tile while the others idle.
constexpr uint32_t SL_BIGRUN = 512;
// big[0, *nbig): the long runs found by the waves; *nbig is 0 on entry and on return
__device__ __forceinline__ void lo_write_runs(uint32_t* __restrict__ sorted, const uint32_t* sv, const uint32_t* n,
                                              const uint32_t* src, const uint32_t* dst, int nb, uint32_t* big,
                                              uint32_t* nbig) {
  // The bucket loop and each run's bounds are wave-uniform: read into scalar registers
  // (readfirstlane), so the loop control and the run's base addresses are scalar work and a run of
  // ~60 entries costs a few VALU (a lane-index compare and two offsets) instead of ~25 of per-bucket
  // set-up in vector registers.
  const uint32_t tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  for (uint32_t b = wave; b < (uint32_t)nb; b += SL_THREADS / 64) {
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(n[b]);
    if (cnt > SL_BIGRUN) {
      if (lane == 0) big[atomicAdd(nbig, 1u)] = b;
      continue;
    }
    const uint32_t s0 = __builtin_amdgcn_readfirstlane(src[b]), d0 = __builtin_amdgcn_readfirstlane(dst[b]);
    const uint32_t* __restrict__ from = sv + s0;
    uint32_t* __restrict__ to = sorted + d0;
#pragma unroll 1
    for (uint32_t i = 0; i < cnt; i += 64) {
      if (i + lane < cnt) to[i + lane] = from[i + lane];
    }
  }
  __syncthreads();
  const uint32_t nbg = *nbig;
  for (uint32_t k = 0; k < nbg; k++) {
    const uint32_t b = big[k], cnt = n[b], s0 = src[b], d0 = dst[b];
    for (uint32_t i = tid; i < cnt; i += SL_THREADS) sorted[d0 + i] = sv[s0 + i];
  }
  __syncthreads();
  if (tid == 0) *nbig = 0;
}

// one block per (partition, chunk): bases from the partition's chunk histograms, then chunk g of
// partition p through LDS in tiles of SL_TILE (one tile unless the partition is skewed past SL_G
// chunks), each bucket's run stored with consecutive lanes (lo_write_runs)
__device__ __forceinline__ void lo_scatter_body(uint32_t* __restrict__ sorted, uint32_t* __restrict__ offsets,
                                                const uint32_t* __restrict__ locnt, const uint32_t* __restrict__ tval,
                                                const uint8_t* __restrict__ tlo, const uint32_t* __restrict__ hi_off,
                                                const uint32_t* __restrict__ cpre, const uint32_t* __restrict__ bpart,
                                                int NH, int lob) {
  __shared__ uint32_t cur[256], tcnt[256], toff[256], big[256];
  __shared__ uint32_t sv[SL_TILE];
  __shared__ uint32_t nbig;
  if (threadIdx.x == 0) nbig = 0;
  uint32_t p, g, G, s0, s1;
  if (!chunk_of_block(cpre, hi_off, bpart, NH, blockIdx.x, p, g, G, s0, s1)) return;  // uniform per block
  const uint32_t tid = threadIdx.x;
  const int nb = 1 << lob;
  // global base of each lo in this chunk: partition start + entries of smaller lo (all chunks) +
  // entries of this lo in earlier chunks; the chunk-0 block publishes the bucket offsets. The chunk's
  // own counts (k_lo_count) give its LDS tile offsets up front.
  __shared__ uint32_t ccnt[256], coff[256];
  uint32_t pref = 0;
  if ((int)tid < nb) {
    const uint32_t* row = locnt + ((uint64_t)p * nb + tid) * SL_G;
    uint32_t tot = 0;
    for (uint32_t q = 0; q < G; q++) {
      const uint32_t v = row[q];
      pref += q < g ? v : 0u;
      ccnt[tid] = q == g ? v : ccnt[tid];
      tot += v;
    }
    tcnt[tid] = tot;
  }
  __syncthreads();
  if (tid < 64) wave_excl_scan256(tcnt, toff, nb);
  else if (tid < 128) wave_excl_scan256(ccnt, coff, nb);
  __syncthreads();
  if ((int)tid < nb) {
    const uint32_t base = s0 + toff[tid];
    if (g == 0) offsets[((uint32_t)p << lob) + tid + 1] = base;
    cur[tid] = base + pref;
    toff[tid] = coff[tid];  // slot cursor of lo in the LDS tile
  }
  uint32_t c0, c1;
  chunk_range(s0, s1, G, g, c0, c1);
  if (c1 - c0 <= (uint32_t)SL_TILE) {
    // the chunk is one tile (every partition of a non-skewed MSM): each entry goes straight to its
    // slot (slot cursor per lo), then each bucket's run leaves with consecutive lanes
    __syncthreads();
    // every entry's lo and value loaded first (all loads in flight at once), then the slot atomics
    constexpr int PER = SL_TILE / SL_THREADS;
    uint32_t lo_k[PER], val_k[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t e = c0 + tid + k * SL_THREADS;
      if (e < c1) {
        lo_k[k] = tlo[e];
        val_k[k] = tval[e];
      }
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t e = c0 + tid + k * SL_THREADS;
      if (e < c1) sv[atomicAdd(&toff[lo_k[k]], 1u)] = val_k[k];
    }
    __syncthreads();
    lo_write_runs(sorted, sv, ccnt, coff, cur, nb, big, &nbig);
    return;
  }
  for (uint32_t t0 = c0; t0 < c1; t0 += SL_TILE_BIG) {
    const uint32_t tn = c1 - t0 < (uint32_t)SL_TILE_BIG ? c1 - t0 : (uint32_t)SL_TILE_BIG;
    __syncthreads();
    if ((int)tid < nb) tcnt[tid] = 0;
    __syncthreads();
    // per entry (rank within its bucket << 8) | lo in one register; the values are loaded after the
    // scan straight into their LDS slots (this path: skewed partitions only; the kernel stays within
    // 64 VGPRs, two 1024-thread blocks per CU, without scratch)
    uint32_t rl[SL_TILE_BIG / SL_THREADS];
#pragma unroll
    for (int k = 0; k < SL_TILE_BIG / SL_THREADS; k++) {
      const uint32_t e = tid + k * SL_THREADS;
      if (e < tn) {
        const uint32_t l = tlo[t0 + e];
        rl[k] = (atomicAdd(&tcnt[l], 1u) << 8) | l;
      }
    }
    __syncthreads();
    if (tid < 64) wave_excl_scan256(tcnt, toff, nb);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SL_TILE_BIG / SL_THREADS; k++) {
      const uint32_t e = tid + k * SL_THREADS;
      if (e < tn) sv[toff[rl[k] & 255u] + (rl[k] >> 8)] = tval[t0 + e];
    }
    __syncthreads();
    lo_write_runs(sorted, sv, tcnt, toff, cur, nb, big, &nbig);
    __syncthreads();
    if ((int)tid < nb) cur[tid] += tcnt[tid];
  }
}

#ifdef KGS_DIAG_CLOCK
// diagnostic builds only: every k_lo_scatter block appends {offsets pointer (the MSM's context),
// real-time counter at block start and end, CU id | block index << 32} to a ring, to see how long the
// workgroups sit resident and when they start relative to each other, alone and in flight
// (profiles/lo_residency.py; VERDICT r3 Next #4)
constexpr uint32_t KGS_LOREC_CAP = 1u << 16;
__device__ unsigned long long g_kgs_lorec[4 * KGS_LOREC_CAP];
__device__ unsigned int g_kgs_lorec_n;
#endif

__global__ void __launch_bounds__(SL_THREADS) __attribute__((amdgpu_waves_per_eu(KGS_SL_WPE, 8))) k_lo_scatter(uint32_t* __restrict__ sorted, uint32_t* __restrict__ offsets,
                                                           const uint32_t* __restrict__ locnt,
                                                           const uint32_t* __restrict__ tval,
                                                           const uint8_t* __restrict__ tlo,
                                                           const uint32_t* __restrict__ hi_off,
                                                           const uint32_t* __restrict__ cpre,
                                                           const uint32_t* __restrict__ bpart, int NH, int lob) {
  KGS_AUX_PRIO();
#ifdef KGS_DIAG_CLOCK
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  lo_scatter_body(sorted, offsets, locnt, tval, tlo, hi_off, cpre, bpart, NH, lob);
#ifdef KGS_DIAG_CLOCK
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t slot = atomicAdd(&g_kgs_lorec_n, 1u) % KGS_LOREC_CAP;
    unsigned long long* o = g_kgs_lorec + 4 * slot;
    o[0] = (unsigned long long)(uintptr_t)offsets;
    o[1] = rt0;
    o[2] = rt1;
    o[3] = (unsigned long long)__smid() | ((unsigned long long)blockIdx.x << 32);
  }
#endif
}

// ------------------------------------------------------------------ bucket accumulation
constexpr uint32_t CB_T = 16;  // partials per thread per combine level
constexpr int CB_LEVELS = 3;

// Segment s (first run inside bucket [o0, o1)) starts a level chunk of `stride` partials x CB_T
// when its bucket has more than CB_T partials and s is aligned: append it to that level's list.
__device__ __forceinline__ void combine_enqueue(uint32_t* list, uint32_t* cnt, uint64_t s, uint64_t o0, uint64_t o1,
                                                uint32_t L, uint64_t stride) {
  if (s * L <= o0) return;  // the segment's first run starts its bucket (run_rec b), not a partial
  const uint64_t s_lo = o0 / L + 1, s_hi = (o1 + L - 1) / L;
  if (s_hi - s_lo <= CB_T) return;  // short list: summed directly by k_combine
  if ((s - s_lo) % (stride * CB_T) != 0 || s + stride >= s_hi) return;
  list[atomicAdd(cnt, 1u)] = (uint32_t)s;
}

// Run records (g1_acc29 raw form, RAW29_WORDS words each) of one MSM live in ONE array `raw`:
// record b < nbins = B + 1 is the run that starts bucket b (later overwritten by the bucket's
// total), record nbins + s the partial of segment s (a run that started before the segment).
__device__ __forceinline__ uint32_t* run_rec(uint32_t* raw, uint64_t i) { return raw + RAW29_WORDS * i; }
__device__ __forceinline__ const uint32_t* run_rec(const uint32_t* raw, uint64_t i) { return raw + RAW29_WORDS * i; }

// Blocks of 256 per CU in the bucket accumulation (= waves per SIMD). 3 fits the 166-VGPR add loop
// and is 2.5 % faster for one MSM alone; 2 leaves a third of every register file to the kernels of
// the other proofs in flight and of the second MSM lane: +0.7 % proofs/s and 15.6 -> 14.8 ms
// single-proof latency (same-box A/B, 128-proof runs).
#ifndef KGS_ACC_WAVES
#define KGS_ACC_WAVES 2
#endif
// Register budget of the add loop (template VW): the default build is compiled for 3 waves/SIMD
// (<= 168 VGPRs) although launched at KGS_ACC_WAVES, so two resident accumulate waves leave 176 of a
// SIMD's 512 VGPRs and the other in-flight proofs' kernels of up to 176 VGPRs (the MSM tail's
// combine levels at 162, NTT passes, divisions) co-reside instead of waiting for a whole accumulate
// launch to drain: +1.9 % proofs/s (same-box A/B). A context running two MSM lanes uses the VW = 2
// build, which reserves 176 VGPRs (v175 is clobbered, whatever the compiler needs): two waves then
// take a SIMD's whole register file, its second lane's accumulation waits for the first instead of
// co-running with it (its blocks start as the first lane's finish), and the first lane's tail runs
// beside the second lane's accumulation (single-proof latency 16.0 -> 14.8 ms; ordering the two
// accumulations with events instead measured 15.2-16.5 ms: no block-level hand-over).
// diagnostic builds only (wrong results): KGS_DIAG_GATHER_MASK confines the point gathers to a small,
// cache-resident part of the table, to measure what the random HBM gathers cost the add loop
#ifndef KGS_DIAG_GATHER_MASK
#define KGS_DIAG_GATHER_MASK 0x7fffffffu
#endif
#ifdef KGS_DIAG_CLOCK
// diagnostic builds only (-DKGS_DIAG_CLOCK; never the shipped library): thread 0 of each of the first
// KGS_CLK_BLOCKS blocks stamps the shader clock (s_memtime) and the 100 MHz real-time counter
// (s_memrealtime) around its add loop; the last launch's stamps give the clock the chip held while it
// ran (kgs_diag_clock), also with other proofs' kernels in flight. Stamps go to their own buffer.
constexpr int KGS_CLK_BLOCKS = 8192;
__device__ unsigned long long g_kgs_clk[4 * KGS_CLK_BLOCKS];
__device__ unsigned int g_kgs_clk_cu[KGS_CLK_BLOCKS];
#endif
template <int VW>
__global__ void __launch_bounds__(256, VW) k_accumulate(uint32_t* __restrict__ segowner,
                                                    uint32_t* __restrict__ chunklist, uint32_t* __restrict__ chunkcnt,
                                                    const uint32_t* __restrict__ sorted,
                                                    const uint32_t* __restrict__ offsets, uint32_t nbins,
                                                    const uint32_t* __restrict__ table, uint32_t L,
                                                    uint32_t* __restrict__ raw, uint32_t prio_m1, uint32_t prio_m2) {
  if (VW == 2) asm volatile("; reserve v175 (176 VGPRs: two waves per SIMD)" ::: "v175");
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t E = offsets[nbins];
  const uint64_t start = s * L;
  if (start >= E) return;
#ifdef KGS_DIAG_CLOCK
  unsigned long long clk0 = 0, rt0 = 0;
  if (threadIdx.x == 0) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
#endif
  const uint64_t end = start + L < E ? start + L : E;
  // largest b with offsets[b] <= start (offsets nondecreasing, offsets[0] == 0)
  uint32_t lo = 0, hi = nbins;  // invariant offsets[lo] <= start < offsets[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= start) lo = mid; else hi = mid;
  }
  uint32_t b = lo;
  const uint32_t o0 = offsets[b], o1 = offsets[b + 1];
  segowner[s] = b;  // bucket of the segment's first run (read by the combine levels)
  combine_enqueue(chunklist, chunkcnt, s, o0, o1, L, 1);
  g1_acc29 acc;
  acc.set_inf();
  // entry indices fit 32 bits (offsets[] is uint32): fewer live VGPRs in the add loop
  const uint32_t end32 = (uint32_t)end, last = end32 - 1;
  // record of the current run: b if it starts its bucket, nbins + s for the segment's first run when
  // the segment starts inside the bucket (every later run starts at a bucket boundary)
  uint32_t rec = (uint32_t)start == o0 ? b : nbins + (uint32_t)s;
  // bucket ends: bend32 of bucket b and bnext of bucket b + 1, re-read after every entry (a 4-byte
  // cache hit, first needed at the next crossing), so a crossing (some lane of the wave makes one in
  // about half of the iterations at 2^20 points) waits on no load; only empty buckets read offsets[]
  // on the spot
  uint32_t bend32 = o1, bnext = offsets[b + 2 <= nbins ? b + 2 : nbins];
  // software pipeline: the point of entry e+1 and the index of entry e+2 are loaded while entry e is
  // added, UNCONDITIONALLY (indices clamped to the segment's last entry): a conditional prefetch is
  // merged into the loop-carried registers by copies placed right after the loads, and the copies made
  // the wave wait for the gathers it had just issued; here the copies sit at the loop latch, after
  // the add
  uint32_t v = sorted[start];
  uint32_t vn = sorted[start + 1 <= last ? start + 1 : last];
  const uint4* pt = reinterpret_cast<const uint4*>(table + 16 * (uint64_t)(v & KGS_DIAG_GATHER_MASK));
  uint4 a0 = pt[0], a1 = pt[1], a2 = pt[2], a3 = pt[3];
  // Progress priority (prio_m1 != 0): a SIMD's VALU goes to the oldest of its ready waves at equal
  // priority, so of two accumulate waves with the same L entries the older finishes first and the
  // younger then runs alone, without a partner to hide its latencies (alone on the GPU: the earlier
  // block of a CU finishes at ~57 % of the launch, profiles/acc_residency.py). Each wave lowers its
  // priority 2 -> 1 -> 0 after prio_m1 and prio_m2 entries, so a wave that is a level behind is issued
  // first; the late second step leaves little work for the last, equal-priority stretch, after which
  // the younger wave runs alone. The aux kernels run at 3, above every accumulate wave.
  uint32_t it = 0;
  if (prio_m1) __builtin_amdgcn_s_setprio(2);
  for (uint32_t e = (uint32_t)start; e <= last; e++, it++) {
    if (it == prio_m1) __builtin_amdgcn_s_setprio(1);
    if (it == prio_m2) __builtin_amdgcn_s_setprio(0);
    const uint4* pn = reinterpret_cast<const uint4*>(table + 16 * (uint64_t)(vn & KGS_DIAG_GATHER_MASK));
    const uint4 n0 = pn[0], n1 = pn[1], n2 = pn[2], n3 = pn[3];
    const uint32_t vnn = sorted[e + 2 <= last ? e + 2 : last];
    if (e >= bend32) {
      acc.store_raw(run_rec(raw, rec));
      b++;
      bend32 = bnext;
      while (e >= bend32) {  // empty buckets
        b++;
        bend32 = offsets[b + 1];
      }
      rec = b;
      acc.set_inf();
    }
    bnext = offsets[b + 2 <= nbins ? b + 2 : nbins];
    const uint32_t xw[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const uint32_t yw[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
    acc.add_aff(xw, yw, (v & 0x80000000u) != 0);
    a0 = n0; a1 = n1; a2 = n2; a3 = n3;
    v = vn;
    vn = vnn;
  }
  acc.store_raw(run_rec(raw, rec));
#ifdef KGS_DIAG_CLOCK
  if (threadIdx.x == 0 && blockIdx.x < KGS_CLK_BLOCKS) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o = g_kgs_clk + 4 * blockIdx.x;
    o[0] = clk0;
    o[1] = clk1;
    o[2] = rt0;
    o[3] = rt1;
    unsigned int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_kgs_clk_cu[blockIdx.x] = ((xcc & 15u) << 16) | (unsigned int)__smid();
  }
#endif
}

#ifdef KGS_DIAG_CLOCK
// k_lo_scatter block records (oldest first when the ring has not wrapped); reset = 1 clears the ring
extern "C" int kgs_diag_lorec(unsigned long long* out, unsigned int cap, unsigned int* n, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  unsigned int cnt = 0;
  if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(g_kgs_lorec_n), sizeof(cnt)) != hipSuccess) return 1;
  const unsigned int have = cnt < KGS_LOREC_CAP ? cnt : KGS_LOREC_CAP;
  const unsigned int m = have < cap ? have : cap;
  if (m && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kgs_lorec), 32ull * m) != hipSuccess) return 1;
  *n = m;
  if (reset) {
    const unsigned int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_kgs_lorec_n), &z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}

// median over the stamped blocks of d(shader clock) / d(real time) x 100 MHz, in GHz
// raw stamps of the last accumulate launch: per block {clk0, clk1, rt0, rt1, cu}; returns the count
extern "C" int kgs_diag_clock_raw(unsigned long long* out, int max) {
  static unsigned long long h[4 * KGS_CLK_BLOCKS];
  static unsigned int cu[KGS_CLK_BLOCKS];
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_kgs_clk), sizeof(h)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(cu, HIP_SYMBOL(g_kgs_clk_cu), sizeof(cu)) != hipSuccess) return -1;
  int n = 0;
  for (int b = 0; b < KGS_CLK_BLOCKS && n < max; b++) {
    if (!(h[4 * b + 3] > h[4 * b + 2])) continue;
    for (int k = 0; k < 4; k++) out[5 * n + k] = h[4 * b + k];
    out[5 * n + 4] = cu[b];
    n++;
  }
  return n;
}

extern "C" int kgs_diag_clock(double* ghz, int* nblocks) {
  static unsigned long long h[4 * KGS_CLK_BLOCKS];
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_kgs_clk), sizeof(h)) != hipSuccess) return 1;
  std::vector<double> v;
  for (int b = 0; b < KGS_CLK_BLOCKS; b++)
    if (h[4 * b + 3] > h[4 * b + 2] && h[4 * b + 1] > h[4 * b]) v.push_back((double)(h[4 * b + 1] - h[4 * b]) / (double)(h[4 * b + 3] - h[4 * b + 2]) * 0.1);
  *nblocks = (int)v.size();
  if (v.empty()) return 1;
  std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
  *ghz = v[v.size() / 2];
  const unsigned long long zero[4 * 64] = {};
  for (int b = 0; b < KGS_CLK_BLOCKS; b += 64) hipMemcpyToSymbol(HIP_SYMBOL(g_kgs_clk), zero, sizeof(zero), 8 * 4 * b);
  return 0;
}
#endif

// Bucket totals. Bucket b = its start record (run_rec b) + the partials of the segments whose start
// lies strictly inside it: segments s_lo(b) = offsets[b]/L + 1 .. s_hi(b) = ceil(offsets[b+1]/L) - 1.
// Buckets can be arbitrarily skewed (a selector polynomial has all-equal coefficients, so every point
// lands in the same bucket of each window), so the partials are first reduced in CB_LEVELS chunked
// levels: at level j the thread of segment s = s_lo + i*CB_T^(j+1) adds the CB_T partials at stride
// CB_T^j that follow it (in place). The final pass then has <= ceil(m / CB_T^CB_LEVELS) partials per
// bucket, walked by one lane (KGS_COMBINE_LANES). Depth for m partials:
// ~CB_T*CB_LEVELS + m/CB_T^3. Lists of <= CB_T partials (every bucket of a uniform scalar
// distribution) skip the levels. All of the tail (combine, bit sums) adds run records in the fq29
// form with g1_acc29::add; only the c bit sums leave as 256-bit XYZZ points for the host.
__device__ __forceinline__ g1_acc29 shfl_xor_acc(const g1_acc29& a, int mask) {
  g1_acc29 r;
#pragma unroll
  for (int j = 0; j < 9; j++) {
    r.X.l[j] = __shfl_xor(a.X.l[j], mask);
    r.Y.l[j] = __shfl_xor(a.Y.l[j], mask);
    r.ZZ.l[j] = __shfl_xor(a.ZZ.l[j], mask);
    r.ZZZ.l[j] = __shfl_xor(a.ZZZ.l[j], mask);
  }
  r.inf = __shfl_xor((int)a.inf, mask) != 0;
  return r;
}

// level j: one thread per listed chunk start s (stride CB_T^j): add the CB_T - 1 partials that follow
// at that stride, store in place, and list s for level j + 1 if it starts a chunk there
__global__ void __launch_bounds__(256) k_combine_level(uint32_t* __restrict__ raw, uint32_t nbins,
                                                       const uint32_t* __restrict__ segowner,
                                                       const uint32_t* __restrict__ offsets,
                                                       const uint32_t* __restrict__ list_in,
                                                       const uint32_t* __restrict__ cnt_in,
                                                       uint32_t* __restrict__ list_out, uint32_t* __restrict__ cnt_out,
                                                       uint32_t L, uint64_t stride) {
  KGS_AUX_PRIO();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= *cnt_in) return;
  const uint64_t s = list_in[t];
  const uint32_t b = segowner[s];
  const uint64_t o0 = offsets[b], o1 = offsets[b + 1];
  const uint64_t s_hi = (o1 + L - 1) / L;
  const uint64_t top = s + stride * CB_T < s_hi ? s + stride * CB_T : s_hi;
  g1_acc29 acc = g1_acc29::load_raw(run_rec(raw, nbins + s));
  for (uint64_t u = s + stride; u < top; u += stride) acc.add(g1_acc29::load_raw(run_rec(raw, nbins + u)));
  acc.store_raw(run_rec(raw, nbins + s));
  if (list_out) combine_enqueue(list_out, cnt_out, s, o0, o1, L, stride * CB_T);
}

// bucket b's total replaces its start record (run_rec b), for every b in 1..B (empty: infinity).
// KGS_COMBINE_LANES threads per bucket: one thread walks the bucket's partials (1, default), or two
// split them and add their sums with one shuffle (2). A bucket has 2-3 partials at 2^20 points; two
// lanes ran ~6 wave-adds per 64 buckets against ~4 for one lane: +0.7 % proofs/s in 3 of 3 same-box
// reps, combine 0.057 -> 0.053 ms alone, skewed MSMs unchanged (profiles/r04/comb/).
#ifndef KGS_COMBINE_LANES
#define KGS_COMBINE_LANES 1
#endif
constexpr uint32_t COMBINE_LANES = KGS_COMBINE_LANES;
static_assert(COMBINE_LANES == 1 || COMBINE_LANES == 2, "k_combine lanes per bucket");
__global__ void __launch_bounds__(256) k_combine(uint32_t* __restrict__ raw, uint32_t nbins,
                                                 const uint32_t* __restrict__ offsets, uint32_t B, uint32_t L,
                                                 uint64_t stride) {
  KGS_AUX_PRIO();
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = g / COMBINE_LANES + 1;  // buckets 1..B
  const uint32_t sub = g % COMBINE_LANES;
  if (COMBINE_LANES == 1 && b > B) return;
  g1_acc29 acc;
  acc.set_inf();
  if (b <= B) {
    const uint64_t o0 = offsets[b], o1 = offsets[b + 1];
    if (o1 > o0) {
      if (sub == 0) acc = g1_acc29::load_raw(run_rec(raw, b));
      const uint64_t s_lo = o0 / L + 1, s_hi = (o1 + L - 1) / L;
      const uint64_t st = s_hi > s_lo + CB_T ? stride : 1;  // reduced by the levels, or short
      for (uint64_t sgm = s_lo + sub * st; sgm < s_hi; sgm += COMBINE_LANES * st)
        acc.add(g1_acc29::load_raw(run_rec(raw, nbins + sgm)));
    }
  }
  if (COMBINE_LANES == 2) acc.add(shfl_xor_acc(acc, 1));
  if (b <= B && sub == 0) acc.store_raw(run_rec(raw, b));
}

// ------------------------------------------------------------------ sum_b b*S_b via bit sums
// Write a bucket index b < B = 2^(c-1) as b = hi*2^l + lo (l = ceil((c-1)/2) low bits, h = c-1-l
// high bits). Then sum_{b<B} b*S_b = 2^l * sum_hi hi*Row_hi + sum_lo lo*Col_lo with the row sums
// Row_hi = sum_lo S_{hi,lo} and column sums Col_lo = sum_hi S_{hi,lo}, and each of those is a bit sum:
// sum_hi hi*Row_hi = sum_j 2^j TR_j, TR_j = sum_{hi with bit j} Row_hi (likewise TC_k). Hence the c
// bit sums the host's Horner step expects are T_k = TC_k (k < l), T_{l+j} = TR_j (j < h) and
// T_{c-1} = S_B. Work: 2B adds for the row/column sums + c*2^(l-1) for the bit sums (c = 17: 0.13 M
// adds instead of the (c-1)*B/2 = 0.52 M of summing every bucket once per set bit), at the minimal
// depth of log2(B/2) + 1 dependent adds.
// k_rowcol: block r < 2^h sums row r, block 2^h + r sums column r; one element per thread, LDS tree.
__device__ __forceinline__ g1_acc29 block_tree_sum(g1_acc29 v, uint32_t* lds) {
  for (int stride = blockDim.x >> 1; stride > 0; stride >>= 1) {
    if ((int)threadIdx.x >= stride && (int)threadIdx.x < 2 * stride)
      v.store_raw(lds + RAW29_WORDS * (threadIdx.x - stride));
    __syncthreads();
    if ((int)threadIdx.x < stride) v.add(g1_acc29::load_raw(lds + RAW29_WORDS * threadIdx.x));
    __syncthreads();
  }
  return v;
}

__global__ void __launch_bounds__(256) k_rowcol(uint32_t* __restrict__ rc, const uint32_t* __restrict__ raw, int c) {
  KGS_AUX_PRIO();
  __shared__ __attribute__((aligned(16))) uint32_t lds[128 * RAW29_WORDS];
  const int l = c / 2, h = c - 1 - l;  // l = ceil((c-1)/2)
  const uint32_t r = blockIdx.x, t = threadIdx.x;
  const bool row = r < (1u << h);
  g1_acc29 v;
  v.set_inf();
  const uint32_t n = row ? 1u << l : 1u << h;  // elements of this row / column (up to 1024 at c = 20)
  for (uint32_t e = t; e < n; e += 256) {       // more than 256: each thread first sums its share
    const uint32_t b = row ? (r << l) | e : (e << l) | (r - (1u << h));
    if (b) v.add(g1_acc29::load_raw(run_rec(raw, b)));
  }
  v = block_tree_sum(v, lds);
  if (t == 0) v.store_raw(rc + (uint64_t)RAW29_WORDS * r);
}

// The same row / column sums with 16 lanes per line (4 lines per wave): each lane adds its 1/16 of
// the line sequentially, then 4 xor-shuffle levels. 4.75 wave-adds per line instead of the block
// tree's 9 (whose levels leave most lanes of their waves idle), at 19 dependent adds instead of 9:
// the in-flight build (other proofs fill the latency); one proof at a time keeps k_rowcol.
constexpr uint32_t RC_LANES = 16;
__global__ void __launch_bounds__(256) k_rowcol16(uint32_t* __restrict__ rc, const uint32_t* __restrict__ raw, int c) {
  KGS_AUX_PRIO();
  const int l = c / 2, h = c - 1 - l;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t line = gid / RC_LANES, j = gid % RC_LANES;
  const uint32_t nlines = (1u << h) + (1u << l);
  const bool row = line < (1u << h);
  const uint32_t n = row ? 1u << l : 1u << h;  // elements of this row / column (<= 256)
  g1_acc29 v;
  v.set_inf();
  if (line < nlines) {
    for (uint32_t t = j; t < n; t += RC_LANES) {
      const uint32_t b = row ? (line << l) | t : (t << l) | (line - (1u << h));
      if (b) v.add(g1_acc29::load_raw(run_rec(raw, b)));
    }
  }
#pragma unroll
  for (int m = RC_LANES / 2; m >= 1; m >>= 1) v.add(shfl_xor_acc(v, m));  // every lane of the wave
  if (line < nlines && j == 0) v.store_raw(rc + (uint64_t)RAW29_WORDS * line);
}

// one block per k < c: T_k = sum of the column sums with bit k set (k < l), of the row sums with bit
// k - l set (l <= k < c-1), or S_B (k = c-1); 256-bit XYZZ out for the host
__global__ void __launch_bounds__(128) k_bitsum_rc(uint32_t* __restrict__ T, const uint32_t* __restrict__ rc,
                                                   const uint32_t* __restrict__ raw, int c) {
  KGS_AUX_PRIO();
  __shared__ __attribute__((aligned(16))) uint32_t lds[64 * RAW29_WORDS];
  const int l = c / 2, h = c - 1 - l;
  const int k = blockIdx.x;
  const uint32_t t = threadIdx.x;
  g1_acc29 v;
  v.set_inf();
  if (k == c - 1) {
    if (t == 0) v = g1_acc29::load_raw(run_rec(raw, 1u << (c - 1)));
  } else {
    const int bits = k < l ? l : h, j = k < l ? k : k - l;  // sum over 2^(bits-1) entries (512 at c = 20)
    const uint32_t base = k < l ? 1u << h : 0u;             // column sums follow the row sums
    for (uint32_t e = t; e < (1u << (bits - 1)); e += 128) {
      const uint32_t idx = ((e >> j) << (j + 1)) | (1u << j) | (e & ((1u << j) - 1));
      v.add(g1_acc29::load_raw(rc + (uint64_t)RAW29_WORDS * (base + idx)));
    }
  }
  v = block_tree_sum(v, lds);
  if (t == 0) v.to_xyzz().store(T + 32 * (uint64_t)k);
}

// ------------------------------------------------------------------ driver (device part)
void msm_run(hipStream_t st, const MsmTables& tb, MsmWork& w, const uint32_t* scalars, uint64_t N,
             uint32_t* T_out, hipEvent_t* ev, uint64_t pbase, uint64_t pstride, bool exclusive_acc) {
  // ev (optional, 5 events): [0] start, [1] after digits+sort, [2] after k_accumulate,
  // [3] after combine, [4] after bit-sum reduction
  if (ev) hipEventRecord(ev[0], st);
  const int c = tb.c, W = tb.W;
  const uint32_t B = 1u << (c - 1);
  // LOB bits of (key - 1) are sorted inside a partition (<= 8: tlo is a byte), the rest select one
  // of NH = B >> LOB partitions (<= 256 up to c = 17, 2^(c-9) <= NH_MAX above)
  const int lob = msm_lob(c);
  const int NH = (int)(B >> lob);
  const uint32_t nblk = (uint32_t)((N + 256 * SORT_SPT - 1) / (256 * SORT_SPT));
  uint32_t* ptot = w.counts;                  // NH partition totals
  uint32_t* hi_off = w.cursor;                // NH + 1
  uint32_t* cpre = w.cursor + NH_MAX + 8;     // NH + 1: lo-pass chunks per partition, exclusive scan
  uint32_t* bpart = w.cursor + 2 * (NH_MAX + 8);  // lo-pass block -> partition
  uint32_t* bh = w.blockhist;                 // NH x nblk
  const size_t part_lds = (size_t)256 * SORT_SPT * W * 7 + (size_t)12 * NH;
  // the scalars' standard forms (32 B each) go through w.sorted between the two sort passes: only the
  // lo pass writes it later, and it holds E = N * W >= 8 N words (W >= 9 for c <= 31)
  uint32_t* scal_std = w.sorted;
  switch (c) {
#define KGS_SORT_C(CC)                                                                                         \
  case CC:                                                                                                      \
    hipLaunchKernelGGL(k_sort_hist<CC>, dim3(nblk), dim3(256), 0, st, bh, scalars, N, lob, NH, nblk, scal_std); \
    hipLaunchKernelGGL(k_sort_scan_blocks, dim3(NH), dim3(256), 0, st, bh, ptot, nblk);                       \
    hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(256), 0, st, hi_off, ptot, NH, w.offsets, B, cpre, bpart); \
    hipLaunchKernelGGL(k_sort_part<CC>, dim3(nblk), dim3(256), part_lds, st, (uint32_t*)w.digit, w.lo, bh,   \
                       ptot, hi_off, scal_std, N, tb.npts, pbase, pstride, lob, NH, nblk);                    \
    break;
    KGS_SORT_C(7) KGS_SORT_C(8) KGS_SORT_C(9) KGS_SORT_C(10) KGS_SORT_C(11) KGS_SORT_C(12)
    KGS_SORT_C(13) KGS_SORT_C(14) KGS_SORT_C(15) KGS_SORT_C(16) KGS_SORT_C(17) KGS_SORT_C(18)
    KGS_SORT_C(19) KGS_SORT_C(20)
#undef KGS_SORT_C
    default:
      return;  // choose_c keeps 7 <= c <= KGS_C_MAX = 20
  }
  // lo-pass grid: an upper bound of sum_p chunk_count(size_p) (blocks past cpre[NH] exit)
  const uint64_t chunk_bound = std::min<uint64_t>((uint64_t)NH * SL_G, NH + N * (uint64_t)W / SL_CHUNK);
  hipLaunchKernelGGL(k_lo_count, dim3((unsigned)chunk_bound), dim3(LC_THREADS), 0, st, w.locnt, w.lo, hi_off, cpre,
                     bpart, NH, lob);
  hipLaunchKernelGGL(k_lo_scatter, dim3((unsigned)chunk_bound), dim3(SL_THREADS), 0, st, w.sorted, w.offsets, w.locnt,
                     (const uint32_t*)w.digit, w.lo, hi_off, cpre, bpart, NH, lob);
  if (ev) hipEventRecord(ev[1], st);
  const uint64_t E = N * (uint64_t)W;  // upper bound of nonzero entries
  // one segment per resident thread (KGS_ACC_WAVES blocks of 256 per CU): every accumulate
  // thread runs once and they all finish together (a second, partial round of blocks would
  // leave most of the chip idle for a whole segment's duration)
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  const uint64_t resident = (uint64_t)cus * KGS_ACC_WAVES * 256;
  uint64_t L = (E + resident - 1) / resident;
  if (L < 4) L = 4;
  if ((E + L - 1) / L > (1ull << 18)) L = (E + (1ull << 18) - 1) >> 18;  // work buffers hold 2^18 + 2^16 segments
  const uint64_t nseg = (E + L - 1) / L;
  // chunk lists of the combine levels: list j holds <= nseg / CB_T^(j+1) + B entries
  uint32_t* cnt = w.chunkcnt;
  const uint64_t lcap = nseg / CB_T + B + 16;
  hipMemsetAsync(cnt, 0, 4 * CB_LEVELS, st);
  // progress priority (k_accumulate): KGS_ACC_PRIO 0 off, 1 the exclusive (two-lane) build, 2 every launch
  static const int acc_prio = [] {
    const char* e = getenv("KGS_ACC_PRIO");
    return e ? atoi(e) : 1;
  }();
  // steps at 3/4 and 93/100 of the segment (a two-wave issue model with the leftover rate of the
  // younger wave measured alone, 0.34 of the older's, puts these within 1 % of the best pair)
#ifdef KGS_NO_PRIO_AUX
  const bool prio = false;  // the A/B build without wave priorities: no step priority either
  (void)acc_prio;
#else
  const bool prio = acc_prio >= 2 || (acc_prio == 1 && exclusive_acc);
#endif
  const uint32_t pm1 = prio ? (uint32_t)(3 * L / 4) : 0u, pm2 = prio ? (uint32_t)(93 * L / 100) : 0u;
  if (exclusive_acc)
    hipLaunchKernelGGL(k_accumulate<2>, dim3(nb(nseg)), dim3(256), 0, st, w.segowner, w.chunklist, cnt, w.sorted,
                       w.offsets, B + 1, tb.table, (uint32_t)L, w.raw29, pm1, pm2);
  else
    hipLaunchKernelGGL(k_accumulate<3>, dim3(nb(nseg)), dim3(256), 0, st, w.segowner, w.chunklist, cnt, w.sorted,
                       w.offsets, B + 1, tb.table, (uint32_t)L, w.raw29, pm1, pm2);
  if (ev) hipEventRecord(ev[2], st);  // the accumulate phase is the k_accumulate launch alone
  uint64_t stride = 1, cap = lcap;
  for (int j = 0; j < CB_LEVELS; j++, stride *= CB_T) {
    uint32_t* lin = w.chunklist + (uint64_t)j * lcap;
    uint32_t* lout = j + 1 < CB_LEVELS ? w.chunklist + (uint64_t)(j + 1) * lcap : nullptr;
    hipLaunchKernelGGL(k_combine_level, dim3(nb(cap)), dim3(256), 0, st, w.raw29, B + 1, w.segowner, w.offsets, lin,
                       cnt + j, lout, lout ? cnt + j + 1 : nullptr, (uint32_t)L, stride);
    cap = cap / CB_T + B + 16;
  }
  hipLaunchKernelGGL(k_combine, dim3(nb(COMBINE_LANES * (uint64_t)B)), dim3(256), 0, st, w.raw29, B + 1, w.offsets, B,
                     (uint32_t)L, stride);
  if (ev) hipEventRecord(ev[3], st);
  // row / column sums (2^h + 2^l blocks), then the c bit sums
  const uint32_t nlines = (1u << (c - 1 - c / 2)) + (1u << (c / 2));
#ifndef KGS_ROWCOL16
#define KGS_ROWCOL16 1
#endif
  if (exclusive_acc || !KGS_ROWCOL16)
    hipLaunchKernelGGL(k_rowcol, dim3(nlines), dim3(256), 0, st, w.part, w.raw29, c);
  else
    hipLaunchKernelGGL(k_rowcol16, dim3((nlines * RC_LANES + 255) / 256), dim3(256), 0, st, w.part, w.raw29, c);
  hipLaunchKernelGGL(k_bitsum_rc, dim3(c), dim3(128), 0, st, T_out, w.part, w.raw29, c);
  if (ev) hipEventRecord(ev[4], st);
}

// ------------------------------------------------------------------ fixed-base (synthetic SRS)
// out[i] = s_i * G with s_i = from_mont(sc[i]); tbl[j*256 + d] = (d * 2^(8j)) G, affine.
__global__ void __launch_bounds__(256) k_fixed_base(uint32_t* __restrict__ out_xyzz, const uint32_t* __restrict__ sc,
                                                    uint64_t count, const uint32_t* __restrict__ tbl) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  fr s = fr::load(sc + 8 * i).from_mont();
  g1_xyzz acc = g1_xyzz::inf();
  for (int j = 0; j < 32; j++) {
    uint32_t d = (s.v[j >> 2] >> ((j & 3) * 8)) & 0xffu;
    if (d) acc.add_aff(g1_aff::load(tbl + 16 * ((uint64_t)j * 256 + d)));
  }
  acc.store(out_xyzz + 32 * i);
}

void launch_fixed_base(hipStream_t st, uint32_t* out_xyzz, const uint32_t* sc, uint64_t count, const uint32_t* tbl) {
  hipLaunchKernelGGL(k_fixed_base, dim3(nb(count)), dim3(256), 0, st, out_xyzz, sc, count, tbl);
}

void launch_batch_affine(hipStream_t st, uint32_t* out_aff, const uint32_t* in_xyzz, uint32_t* scratch, uint64_t npts) {
  hipLaunchKernelGGL(k_batch_affine<32>, dim3(nb((npts + 31) / 32)), dim3(256), 0, st, out_aff, in_xyzz, scratch, npts);
}

}  // namespace kgs
