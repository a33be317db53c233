// voxel.hip — voxel down-sample with trace.
//
// Replaces o3d PointCloud.voxel_down_sample_and_trace(vs, min_bound, max_bound,
// approximate_class=False) + idxmat.max(1) + _select_by_idx
// (reference open3dpypro/PointCloud.py:338-341, :361-362, :185-204;
// processors.py:427-430 VoxelDownsample.cpu_model).
//
// Layout & algorithm (HBM-bound integer work; no MFMA):
//   1. key per point in float64 exactly as Open3D: floor(((double)p - min)/vs).
//   2. voxel table: dense int32 array over the grid box when it is small
//      (<= 2n + 2^20 cells), else an open-addressing hash table on a packed
//      63-bit key.  rep[voxel] = max point index  (= idxmat.max(1)).
//      Dense grids of <= kMaxBuckets buckets (bricks of 2^12..2^13 voxels) are
//      reduced without global atomics: the points are binned by brick
//      (block-local LDS histograms, one global atomic per block and brick to
//      reserve a run), then one workgroup per brick takes the max in an LDS
//      table and writes the brick's slice of the table plus the rep flags.
//      Scattered 4-byte stores/atomics into a table larger than L2 were the
//      cost of the plain dense path (k_voxel_assign_dense + k_voxel_settle).
//   3. flags[rep] = 1, then a flag compaction gives the representatives in
//      ascending index order (= _select_by_idx order) for free.
//   4. trace (optional): voxel_of_point via the compaction prefix, Open3D's
//      (M,8) cubic-id matrix via atomicMax into octant slots.
#include "common.hpp"

namespace o3dx {

constexpr uint64_t kEmpty = ~0ull;
constexpr int kHashBits = 21;
constexpr int kHashOff = 1 << (kHashBits - 1);

struct VoxelGeom {
  double mnx, mny, mnz, vs;
  int nx, ny, nz;
  int kx0 = 0;     // x-key window [kx0, kx0 + nx) of a slab (keys stay those of min_bound)
  double ivs = 0;  // 1 / vs (the binning's multiply; keys stay the division's, voxel_of)
};

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

struct P3 {
  float x, y, z;
};

// Open3D: ref_coord = (p - voxel_min_bound) / voxel_size; voxel_index = floor.
__device__ __forceinline__ void voxel_ref(const P3& q, const VoxelGeom& g, double r[3], int v[3]) {
  r[0] = ((double)q.x - g.mnx) / g.vs;
  r[1] = ((double)q.y - g.mny) / g.vs;
  r[2] = ((double)q.z - g.mnz) / g.vs;
  v[0] = (int)floor(r[0]) - g.kx0;
  v[1] = (int)floor(r[1]);
  v[2] = (int)floor(r[2]);
}

__global__ void __launch_bounds__(kBlock) k_voxel_assign_dense(const float* __restrict__ xyz, int64_t n,
                                                               VoxelGeom g, int32_t* __restrict__ rep,
                                                               int32_t* __restrict__ vid, int* __restrict__ err) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double r[3];
    int v[3];
    voxel_ref(p[i], g, r, v);
    if (v[0] < 0 || v[0] >= g.nx || v[1] < 0 || v[1] >= g.ny || v[2] < 0 || v[2] >= g.nz) {
      *err = 1;
      vid[i] = -1;
      continue;
    }
    int32_t id = v[0] + g.nx * (v[1] + g.ny * v[2]);
    vid[i] = id;
    rep[id] = (int32_t)i;  // plain store: some index of the voxel wins (k_voxel_settle makes it the max)
  }
}

// Second half of the dense assignment: the racy plain stores above left one of
// each voxel's indices in the table; only points with a larger index need the
// (device-scope, slow) atomicMax.  Grid-stride rounds run in index order, so
// the last writer usually is already the maximum and few atomics remain.
__global__ void __launch_bounds__(kBlock) k_voxel_settle(const int32_t* __restrict__ vid, int64_t n,
                                                         int32_t* __restrict__ rep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t id = vid[i];
    if (id >= 0 && rep[id] < (int32_t)i) atomicMax(&rep[id], (int32_t)i);
  }
}

// ------------------------------------------------------- brick-binned path
constexpr int kBinBlock = 512;
constexpr int kBinPer = 32;                    // points per thread in the binning passes
constexpr int kBinChunk = kBinBlock * kBinPer; // points per binning block
constexpr int kMaxBuckets = 4096;              // LDS histogram (16 KB); scatter LDS <= 64 KB
constexpr int kMaxBrickBits = 13;              // LDS max table (32 KB)
constexpr int kReduceBlock = 512;

struct Bricks {
  int sx, sy, sz;     // log2 brick extent per axis
  int nbx, nby, nbz;  // bricks per axis
  int nb;
  int ncp;            // one-pass binning: segment copies per brick
};

// floor(d / vs) through a multiply: q = d * (1/vs) is within |q| 2^-51 of the
// division's correctly rounded quotient, so their floors can only differ
// when an integer lies within that distance of q; those keys (~2^-20 of
// them) take the division.  Bit-identical keys at a third of the f64 work.
__device__ __forceinline__ int voxel_key(double d, double vs, double ivs) {
  const double q = d * ivs;
  const double k = floor(q);
  const double f = q - k;
  const double tol = fabs(q) * 0x1p-50;
  return (int)((f <= tol || f >= 1.0 - tol) ? floor(d / vs) : k);
}

__device__ __forceinline__ bool voxel_of(const P3& q, const VoxelGeom& g, int v[3]) {
  v[0] = voxel_key((double)q.x - g.mnx, g.vs, g.ivs) - g.kx0;
  v[1] = voxel_key((double)q.y - g.mny, g.vs, g.ivs);
  v[2] = voxel_key((double)q.z - g.mnz, g.vs, g.ivs);
  return v[0] >= 0 && v[0] < g.nx && v[1] >= 0 && v[1] < g.ny && v[2] >= 0 && v[2] < g.nz;
}

// (brick << 16) | local voxel within the brick
__device__ __forceinline__ uint32_t brick_code(const int v[3], const Bricks& b) {
  const uint32_t bk = (uint32_t)((v[0] >> b.sx) + b.nbx * ((v[1] >> b.sy) + b.nby * (v[2] >> b.sz)));
  const uint32_t lx = v[0] & ((1 << b.sx) - 1), ly = v[1] & ((1 << b.sy) - 1), lz = v[2] & ((1 << b.sz) - 1);
  return (bk << 16) | lx | (ly << b.sx) | (lz << (b.sx + b.sy));
}

// Pass 1: brick counts per block (LDS histogram); each block reserves its run
// in every brick it touches with one atomic on the brick's total (totals on
// separate 64-B lines), so no scan over (brick, block) is needed: the order of
// the runs inside a brick is the atomics' (the reduce takes a max, which does
// not care).  roff[block * nb + k] = the block's offset inside brick k.  Also
// writes the voxel id per point when the trace needs it.
constexpr int kTotStride = 16;  // int32 per brick total (one 64-B line each)
// One-pass binning: copies of each brick's total, block b reserving in copy
// b % copies (its own slice of the brick's segment).  768 blocks x 614
// bricks of returning atomics on 614 words were serialised per word (C2:
// ~20 us of the kernel's 84); 4 copies cut each word's queue to a quarter.
// (measured round 5 at C2: 1 / 2 / 4 copies within 3 %; 8, one per XCD by
// block % 8, 55 % slower)
__host__ __device__ inline int seg_copies(int nb) { return nb <= kMaxBuckets / 4 ? 4 : nb <= kMaxBuckets / 2 ? 2 : 1; }
constexpr int kMaxCopies = 4;

__global__ void __launch_bounds__(kBinBlock) k_vbin_count(const float* __restrict__ xyz, int64_t n, VoxelGeom g,
                                                       Bricks b, int32_t* __restrict__ roff,
                                                       int32_t* __restrict__ btot, int32_t* __restrict__ vid,
                                                       int* __restrict__ err) {
  __shared__ int32_t hist[kMaxBuckets];
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int k = threadIdx.x; k < b.nb; k += kBinBlock) hist[k] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kBinChunk;
  bool bad = false;
#pragma unroll 4
  for (int j = 0; j < kBinPer; ++j) {
    const int64_t i = base + threadIdx.x + (int64_t)j * kBinBlock;
    if (i >= n) break;
    int v[3];
    const bool in = voxel_of(p[i], g, v);
    if (in) atomicAdd(&hist[brick_code(v, b) >> 16], 1);
    bad |= !in;
    if (vid) vid[i] = in ? v[0] + g.nx * (v[1] + g.ny * v[2]) : -1;
  }
  if (bad) *err = 1;
  __syncthreads();
  for (int k = threadIdx.x; k < b.nb; k += kBinBlock) {
    const int c = hist[k];
    roff[(int64_t)blockIdx.x * b.nb + k] = c ? atomicAdd(&btot[k * kTotStride], c) : 0;
  }
}

// Exclusive scan of the brick totals into LDS base[0..nb] (each thread a span
// of bricks); every scatter block and the reduce recompute it from the totals.
__device__ __forceinline__ void brick_bases(const int32_t* __restrict__ btot, int nb, int32_t* base, int32_t* wsum) {
  const int span = (nb + kBinBlock - 1) / kBinBlock;
  const int k0 = threadIdx.x * span, k1 = min(k0 + span, nb);
  int run = 0;
  for (int k = k0; k < k1; ++k) run += btot[k * kTotStride];
  int tot;
  int ex = block_excl_scan<kBinBlock>(run, wsum, &tot);
  for (int k = k0; k < k1; ++k) {
    base[k] = ex;
    ex += btot[k * kTotStride];
  }
  if (threadIdx.x == 0) base[nb] = tot;
  __syncthreads();
}

// Pass 2: scatter (local << 32 | index) into the block's run of each brick
// (boff = the scanned brick-major histogram).  The block's points go out in
// rounds of kBinRound: sorted by brick in LDS first, so each brick's entries
// leave as one contiguous run (coalesced stores instead of one line per lane).
constexpr int kBinRound = 4096;

// dynamic LDS: stage[kBinRound] (u64), cur[nb], loc[nb + 1]
inline size_t scatter_lds_bytes(int nb) { return kBinRound * sizeof(uint64_t) + (2 * (size_t)nb + 1) * sizeof(int32_t); }

__global__ void __launch_bounds__(kBinBlock) k_vbin_scatter(const float* __restrict__ xyz, int64_t n, VoxelGeom g,
                                                         Bricks b, const int32_t* __restrict__ roff,
                                                         const int32_t* __restrict__ btot,
                                                         int32_t* __restrict__ bbase,
                                                         uint64_t* __restrict__ entries) {
  static_assert(kBinChunk % kBinRound == 0 && kBinRound % kBinBlock == 0, "round shape");
  extern __shared__ uint64_t lds_u64[];
  uint64_t* stage = lds_u64;
  int32_t* cur = reinterpret_cast<int32_t*>(lds_u64 + kBinRound);  // global address of stage slot 0, per brick
  int32_t* loc = cur + b.nb;                                         // round: count -> offset -> cursor
  __shared__ int32_t wsum[kBinBlock / 64 + 1];
  const P3* p = reinterpret_cast<const P3*>(xyz);
  brick_bases(btot, b.nb, loc, wsum);  // loc[] holds the bases until the first round resets it
  for (int k = threadIdx.x; k < b.nb; k += kBinBlock) cur[k] = loc[k] + roff[(int64_t)blockIdx.x * b.nb + k];
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k <= b.nb; k += kBinBlock) bbase[k] = loc[k];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kBinChunk;
  constexpr int kPer = kBinRound / kBinBlock;           // points per thread per round
  const int span = (b.nb + kBinBlock - 1) / kBinBlock;  // bricks per thread in the local scan
  for (int r0 = 0; r0 < kBinChunk && base + r0 < n; r0 += kBinRound) {
    for (int k = threadIdx.x; k < b.nb; k += kBinBlock) loc[k] = 0;
    __syncthreads();
    uint32_t code[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = base + r0 + threadIdx.x + (int64_t)j * kBinBlock;
      int v[3];
      code[j] = ~0u;
      if (i < n && voxel_of(p[i], g, v)) {
        code[j] = brick_code(v, b);
        atomicAdd(&loc[code[j] >> 16], 1);
      }
    }
    __syncthreads();
    // exclusive scan of the round's brick counts (each thread a span of bricks);
    // cur[k] becomes the global address of stage slot 0 for brick k
    const int k0 = threadIdx.x * span, k1 = min(k0 + span, b.nb);
    int run = 0;
    for (int k = k0; k < k1; ++k) run += loc[k];
    int tot;
    int ex = block_excl_scan<kBinBlock>(run, wsum, &tot);
    for (int k = k0; k < k1; ++k) {
      const int c = loc[k];
      loc[k] = ex;
      cur[k] -= ex;
      ex += c;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (code[j] == ~0u) continue;
      const int64_t i = base + r0 + threadIdx.x + (int64_t)j * kBinBlock;
      const int at = atomicAdd(&loc[code[j] >> 16], 1);
      stage[at] = ((uint64_t)(code[j] >> 16) << 48) | ((uint64_t)(code[j] & 0xffffu) << 32) | (uint32_t)i;
    }
    __syncthreads();
    // consecutive stage slots of one brick -> consecutive addresses of its run
    for (int t = threadIdx.x; t < tot; t += kBinBlock) {
      const uint64_t e = stage[t];
      entries[cur[(int)(e >> 48)] + t] = e & 0x0000ffffffffffffull;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < b.nb; k += kBinBlock) cur[k] += loc[k];  // loc[k] = end of brick k's slice
    __syncthreads();
  }
}

// One-pass binning (replaces count + scatter when every brick's entries fit
// a fixed segment of `cap` slots): a block bins its 8192 points by brick in
// LDS, reserves each brick's run with one atomic on the brick's total (the
// run lands at k * cap + offset: no scan over bricks or blocks), and writes
// the runs from the LDS stage.  A brick whose total passes cap drops the
// excess and raises err bit 16: the host reruns with count + scatter.
// FB threads x FP points per thread, one workgroup per CU (measured: two
// 512 x 14 workgroups per CU, 87 us against 77 at C2 — twice the blocks make
// twice the reservation atomics, ~18 us of the kernel)
constexpr int kFusePer = 16;
constexpr int kFuseBlock = 1024;
constexpr int kFuseChunk = kFuseBlock * kFusePer;

// dynamic LDS: stage[FB * FP] (u64), loc[nb + 1], dst[nb]
inline size_t fused_lds_bytes(int nb, int chunk_cap = kFuseChunk) {
  return (size_t)chunk_cap * sizeof(uint64_t) + (2 * (size_t)nb + 1) * sizeof(int32_t);
}

// chunk: points per block (<= kFuseChunk), chosen so the block count is a
// whole number of CU-waves of blocks (fused_grid)
template <int FB, int FP>
__device__ __forceinline__ void vbin_fused_body(const float* __restrict__ xyz, int64_t n, const VoxelGeom& g,
                                                const Bricks& b, int cap, int32_t* __restrict__ btot,
                                                uint64_t* __restrict__ entries, int32_t* __restrict__ vid,
                                                int* __restrict__ err, int chunk) {
  extern __shared__ uint64_t lds_u64[];
  uint64_t* stage = lds_u64;
  int32_t* loc = reinterpret_cast<int32_t*>(lds_u64 + FB * FP);      // count -> offset -> cursor
  int32_t* dst = loc + b.nb + 1;                                      // segment index of stage slot 0, per brick
  __shared__ int32_t wsum[FB / 64 + 1];
  __shared__ int ovf;
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int k = threadIdx.x; k < b.nb; k += FB) loc[k] = 0;
  if (threadIdx.x == 0) ovf = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * chunk;
  const int64_t end = min(base + chunk, n);
  uint32_t code[FP];
  bool bad = false;
  // every load of the chunk first (clamped, unconditional), then the keys
  P3 q[FP];
#pragma unroll
  for (int j = 0; j < FP; ++j) q[j] = p[min(base + threadIdx.x + (int64_t)j * FB, end - 1)];
#pragma unroll
  for (int j = 0; j < FP; ++j) {
    const int64_t i = base + threadIdx.x + (int64_t)j * FB;
    code[j] = ~0u;
    if (i < end) {
      int v[3];
      if (voxel_of(q[j], g, v)) {
        code[j] = brick_code(v, b);
        atomicAdd(&loc[code[j] >> 16], 1);
        if (vid) vid[i] = v[0] + g.nx * (v[1] + g.ny * v[2]);
      } else {
        bad = true;
        if (vid) vid[i] = -1;
      }
    }
  }
  if (bad) *err = 1;
  __syncthreads();
  const int span = (b.nb + FB - 1) / FB;
  const int k0 = threadIdx.x * span, k1 = min(k0 + span, b.nb);
  int run = 0;
  for (int k = k0; k < k1; ++k) run += loc[k];
  int tot;
  int ex = block_excl_scan<FB>(run, wsum, &tot);
  const int ncp = b.ncp, cq = (int)(blockIdx.x & (unsigned)(ncp - 1)), sub = cap / ncp;
  for (int k = k0; k < k1; ++k) {
    const int c = loc[k];
    loc[k] = ex;
    if (c) {
      const int o = atomicAdd(&btot[(k * ncp + cq) * kTotStride], c);
      if (o + c > sub) ovf = 1;
      dst[k] = cq * sub + o - ex;  // slot t of brick k -> k * cap + dst[k] + t
    }
    ex += c;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < FP; ++j) {
    if (code[j] == ~0u) continue;
    const int64_t i = base + threadIdx.x + (int64_t)j * FB;
    const int at = atomicAdd(&loc[code[j] >> 16], 1);
    stage[at] = ((uint64_t)(code[j] >> 16) << 48) | ((uint64_t)(code[j] & 0xffffu) << 32) | (uint32_t)i;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < tot; t += FB) {
    const uint64_t e = stage[t];
    const int k = (int)(e >> 48);
    const int o = dst[k] + t;
    if (o < cap) entries[(int64_t)k * cap + o] = e & 0x0000ffffffffffffull;
  }
  if (threadIdx.x == 0 && ovf) atomicOr(err, 16);
}

template <int FB, int FP>
__global__ void __launch_bounds__(FB) k_vbin_fused(const float* __restrict__ xyz, int64_t n, VoxelGeom g, Bricks b,
                                                   int cap, int32_t* __restrict__ btot, uint64_t* __restrict__ entries,
                                                   int32_t* __restrict__ vid, int* __restrict__ err, int chunk) {
  vbin_fused_body<FB, FP>(xyz, n, g, b, cap, btot, entries, vid, err, chunk);
}

// The one-pass binning's grid: its LDS stage allows one workgroup per CU, so
// the block count is rounded up to whole rounds of kFuseCUs blocks and the
// points are spread evenly over them (10M: 768 blocks of 13,021 points instead
// of 611 of 16,384, whose third round ran on 99 of the 256 CUs).
constexpr int kFuseCUs = 256;
static int fused_grid(int64_t n, unsigned* blocks, int chunk_cap = kFuseChunk, int per_cu = 1) {
  const int64_t nb0 = std::max<int64_t>(1, (n + chunk_cap - 1) / chunk_cap);
  const int64_t nb = (nb0 + kFuseCUs * per_cu - 1) / (kFuseCUs * per_cu) * (kFuseCUs * per_cu);
  const int chunk = (int)std::max<int64_t>(1, (n + nb - 1) / nb);
  *blocks = (unsigned)std::max<int64_t>(1, (n + chunk - 1) / chunk);
  return chunk;
}

// Pass 3: one workgroup per brick: max index per voxel in LDS, then the
// brick's slice of the dense table (-1 = empty) and flags[rep] = 1.
// occ2 (nullable; bricks at least 2 voxels along every axis, so the even-
// aligned 2^3 cells never straddle two bricks): the brick's occupied 2^3
// cells, one atomic per brick (the normals' local-dimension estimate).
__global__ void __launch_bounds__(kReduceBlock) k_vbin_reduce(const uint64_t* __restrict__ entries,
                                                              const int32_t* __restrict__ bbase, int cap,
                                                              const int32_t* __restrict__ btot, VoxelGeom g,
                                                              Bricks b, int32_t* __restrict__ table,
                                                              uint8_t* __restrict__ flags,
                                                              unsigned long long* __restrict__ occ2,
                                                              float4* __restrict__ vox_empty) {
  __shared__ int32_t tab[1 << kMaxBrickBits];
  const int nloc = 1 << (b.sx + b.sy + b.sz);
  for (int k = threadIdx.x; k < nloc; k += kReduceBlock) tab[k] = -1;
  __syncthreads();
  const int bk = blockIdx.x;
  // the brick's entries: its run of the scanned layout, or the filled part
  // of each copy's slice of its fixed segment
  const int ncp = cap ? b.ncp : 1, sub = cap / ncp;
  for (int cq = 0; cq < ncp; ++cq) {
    const int64_t e0 = cap ? (int64_t)bk * cap + (int64_t)cq * sub : bbase[bk];
    const int64_t e1 = cap ? e0 + min(btot[(bk * ncp + cq) * kTotStride], sub) : bbase[bk + 1];
    constexpr int kU = 8;  // entry loads in flight per thread
    for (int64_t e = e0 + threadIdx.x; e < e1; e += (int64_t)kU * kReduceBlock) {
      uint64_t wv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) wv[u] = entries[min(e + (int64_t)u * kReduceBlock, e1 - 1)];
#pragma unroll
      for (int u = 0; u < kU; ++u)  // (a clamped duplicate is harmless for a max)
        atomicMax(&tab[(int)(wv[u] >> 32)], (int32_t)(uint32_t)wv[u]);
    }
  }
  __syncthreads();
  const int bx = bk % b.nbx, by = (bk / b.nbx) % b.nby, bz = bk / (b.nbx * b.nby);
  for (int k = threadIdx.x; k < nloc; k += kReduceBlock) {
    const int x = (bx << b.sx) + (k & ((1 << b.sx) - 1));
    const int y = (by << b.sy) + ((k >> b.sx) & ((1 << b.sy) - 1));
    const int z = (bz << b.sz) + (k >> (b.sx + b.sy));
    if (x >= g.nx || y >= g.ny || z >= g.nz) continue;
    const int32_t r = tab[k];
    const int64_t at = x + (int64_t)g.nx * (y + (int64_t)g.ny * z);
    if (table) table[at] = r;
    if (r >= 0) flags[r] = 1;
    // the kept table's empty slots (k_gather_vox fills the occupied ones)
    else if (vox_empty) vox_empty[at] = make_float4(__int_as_float(-1), __int_as_float(-1), __int_as_float(-1),
                                                     __int_as_float(-1));
  }
  if (occ2) {
    // 2^3 cells of the brick: cell c = (cx, cy, cz) local, voxels outside the
    // grid were never assigned (-1)
    const int csx = b.sx - 1, csy = b.sy - 1, csz = b.sz - 1;
    const int ncell = 1 << (csx + csy + csz);
    unsigned long long c = 0;
    for (int k = threadIdx.x; k < ncell; k += kReduceBlock) {
      const int cx = (k & ((1 << csx) - 1)) * 2, cy = ((k >> csx) & ((1 << csy) - 1)) * 2, cz = (k >> (csx + csy)) * 2;
      bool any = false;
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const int x = cx + (d & 1), y = cy + ((d >> 1) & 1), z = cz + (d >> 2);
        any |= tab[x | (y << b.sx) | (z << (b.sx + b.sy))] >= 0;
      }
      c += any;
    }
    __shared__ unsigned long long sh[kReduceBlock / 64];
    c = wave_sum(c);
    if (lane_id() == 0) sh[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long t = 0;
      for (int w = 0; w < kReduceBlock / 64; ++w) t += sh[w];
      if (t) atomicAdd(occ2, t);
    }
  }
}

// Brick shape: 2^bits voxels, split over the axes by repeatedly doubling the
// axis with the most bricks left; nb = 0 when the grid needs more than
// kMaxBuckets bricks (the plain dense path handles it).
__host__ __device__ static Bricks plan_bricks(int nx, int ny, int nz, int max_buckets = kMaxBuckets) {
  Bricks b{};
  for (int bits = 12; bits <= kMaxBrickBits; ++bits) {
    int sh[3] = {0, 0, 0};
    const int64_t d[3] = {nx, ny, nz};
    for (int it = 0; it < bits; ++it) {
      int best = -1;
      int64_t left = 1;
      for (int a = 0; a < 3; ++a) {
        const int64_t l = (d[a] + (1ll << sh[a]) - 1) >> sh[a];
        if (l > left) {
          left = l;
          best = a;
        }
      }
      if (best < 0) break;
      ++sh[best];
    }
    int64_t nb[3];
    for (int a = 0; a < 3; ++a) nb[a] = (d[a] + (1ll << sh[a]) - 1) >> sh[a];
    const int64_t total = nb[0] * nb[1] * nb[2];
    if (total <= max_buckets) {
      b = Bricks{sh[0], sh[1], sh[2], (int)nb[0], (int)nb[1], (int)nb[2], (int)total, 1};
      return b;
    }
  }
  return b;
}

// The one-pass binning's plan from the bounds, the same function on the host
// and (pre-launched, before the host has the bounds) on the device.
// The one-pass kernel's LDS (128 KB stage + 8 B per brick + statics) fits
// one workgroup per CU up to this many bricks.  2048 admits C4's 50M cloud
// (232^3 voxels: 1800 bricks of 2^13), which at 1536 fell to count +
// scatter (1.24 ms against ~0.4 ms); plan_bricks still prefers 2^12-voxel
// bricks when they fit (C2: 614).
constexpr int kFuseMaxBricks = 2048;
// brick totals: (brick, copy) counters on their own 64-B lines (seg_copies
// keeps bricks x copies <= kMaxBuckets)
constexpr int64_t kTotWords = (int64_t)kMaxBuckets * kTotStride;
static_assert(kFuseMaxBricks * 2 <= kMaxBuckets && kMaxBuckets / 4 * kMaxCopies <= kMaxBuckets, "totals");
static int64_t dense_cap(int64_t n);
static int64_t entries_cap(int64_t n);
__host__ __device__ inline int64_t dense_cap_hd(int64_t n) { return 2 * n + (1 << 20); }
__host__ __device__ inline int64_t entries_cap_hd(int64_t n) { return n + n / 2 + (1 << 20); }

struct BinPlan {
  VoxelGeom g;
  Bricks b;
  int cap;  // segment slots per brick; 0: not the one-pass path
  int ok;
};

__host__ __device__ inline uint64_t geom_key(const VoxelGeom& g, int64_t n) {
  return ((uint64_t)g.nx * 73856093u) ^ ((uint64_t)g.ny * 19349663u) ^ ((uint64_t)g.nz * 83492791u) ^ (uint64_t)n;
}

__host__ __device__ inline void fused_plan(const double mn[3], const double mx[3], double vs, int64_t n, int allow,
                                           uint64_t skip_key, BinPlan* P, uint64_t one_copy_key = ~0ull) {
  P->ok = 0;
  P->cap = 0;
  double dims[3];
  for (int a = 0; a < 3; ++a) dims[a] = floor(fmax(0.0, mx[a] - mn[a]) / vs) + 1.0;
  const double ext = fmax(mx[0] - mn[0], fmax(mx[1] - mn[1], mx[2] - mn[2]));
  const double nvox = dims[0] * dims[1] * dims[2];
  if (!allow || n <= 0 || vs * (double)INT32_MAX < ext || !(nvox <= (double)dense_cap_hd(n))) return;
  VoxelGeom g;
  g.mnx = mn[0];
  g.mny = mn[1];
  g.mnz = mn[2];
  g.vs = vs;
  g.ivs = 1.0 / vs;
  g.nx = (int)dims[0];
  g.ny = (int)dims[1];
  g.nz = (int)dims[2];
  const Bricks b = plan_bricks(g.nx, g.ny, g.nz, kFuseMaxBricks);
  if (b.nb <= 0 || b.nb > kFuseMaxBricks) return;
  const int64_t seg = entries_cap_hd(n) / b.nb;
  const double full = (double)n * (double)(1ll << (b.sx + b.sy + b.sz)) / nvox;
  if (seg > INT32_MAX || !((double)seg >= 1.03 * full + 2048.0) || geom_key(g, n) == skip_key) return;
  P->g = g;
  P->b = b;
  P->b.ncp = geom_key(g, n) == one_copy_key ? 1 : seg_copies(b.nb);
  P->cap = (int)seg;
  P->ok = 1;
}

// The same plan on a given geometry (the slab path's x-key window: g.kx0,
// g.nx = the window's width).
inline void fused_plan_geom(const VoxelGeom& g, int64_t n, int allow, uint64_t skip_key, BinPlan* P,
                            uint64_t one_copy_key = ~0ull) {
  P->ok = 0;
  P->cap = 0;
  const double nvox = (double)g.nx * (double)g.ny * (double)g.nz;
  if (!allow || n <= 0 || !(nvox <= (double)dense_cap_hd(n))) return;
  const Bricks b = plan_bricks(g.nx, g.ny, g.nz, kFuseMaxBricks);
  if (b.nb <= 0 || b.nb > kFuseMaxBricks) return;
  const int64_t seg = entries_cap_hd(n) / b.nb;
  const double full = (double)n * (double)(1ll << (b.sx + b.sy + b.sz)) / nvox;
  if (seg > INT32_MAX || !((double)seg >= 1.03 * full + 2048.0) || geom_key(g, n) == skip_key) return;
  P->g = g;
  P->b = b;
  P->b.ncp = geom_key(g, n) == one_copy_key ? 1 : seg_copies(b.nb);
  P->cap = (int)seg;
  P->ok = 1;
}

// The one-pass binning's plan, computed by the bounds' final kernel
// (k_aabb_final_tail) from the bounds it just folded.
struct PlanTail {
  double vs;
  int64_t n;
  int allow;
  uint64_t skip_key, one_copy_key;
  BinPlan* plan;
  __device__ void operator()(const double* mm) const {
    const double mn[3] = {mm[0], mm[1], mm[2]}, mx[3] = {mm[3], mm[4], mm[5]};
    BinPlan P;
    fused_plan(mn, mx, vs, n, allow, skip_key, &P, one_copy_key);
    *plan = P;
  }
};

template <int FB, int FP>
__global__ void __launch_bounds__(FB) k_vbin_fused_pre(const float* __restrict__ xyz, int64_t n,
                                                       const BinPlan* __restrict__ plan, int32_t* __restrict__ btot,
                                                       uint64_t* __restrict__ entries, int32_t* __restrict__ vid,
                                                       int* __restrict__ err, int chunk) {
  if (!plan->ok) return;
  const VoxelGeom g = plan->g;
  const Bricks b = plan->b;
  vbin_fused_body<FB, FP>(xyz, n, g, b, plan->cap, btot, entries, vid, err, chunk);
}

// launch of the one-pass binning (nb_lds: the bricks its LDS is sized for)
template <bool PRE, class... A>
static void launch_fused(int nb_lds, int64_t n, hipStream_t s, A... args) {
  unsigned nfb;
  const int chunk = fused_grid(n, &nfb);
  if constexpr (PRE)
    hipLaunchKernelGGL((k_vbin_fused_pre<kFuseBlock, kFusePer>), dim3(nfb), dim3(kFuseBlock), fused_lds_bytes(nb_lds),
                       s, args..., chunk);
  else
    hipLaunchKernelGGL((k_vbin_fused<kFuseBlock, kFusePer>), dim3(nfb), dim3(kFuseBlock), fused_lds_bytes(nb_lds), s,
                       args..., chunk);
}

__global__ void __launch_bounds__(kBlock) k_voxel_assign_hash(const float* __restrict__ xyz, int64_t n,
                                                              VoxelGeom g, unsigned long long* __restrict__ keys,
                                                              int32_t* __restrict__ rep, uint32_t tmask,
                                                              int32_t* __restrict__ vid, int* __restrict__ err) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double r[3];
    int v[3];
    voxel_ref(p[i], g, r, v);
    bool bad = false;
    uint64_t key = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      int o = v[a] + kHashOff;
      bad |= (o < 0) | (o >= (1 << kHashBits));
      key |= (uint64_t)(uint32_t)o << (kHashBits * a);
    }
    if (bad) {
      *err = 2;
      vid[i] = 0;
      continue;
    }
    uint32_t s = (uint32_t)mix64(key) & tmask;
    while (true) {
      unsigned long long prev = atomicCAS(&keys[s], (unsigned long long)kEmpty, (unsigned long long)key);
      if (prev == kEmpty || prev == key) break;
      s = (s + 1) & tmask;
    }
    vid[i] = (int32_t)s;
    atomicMax(&rep[s], (int32_t)i);
  }
}

// ------------------------------------------------- hash-binned sparse path
// Grids too large for a dense table (sparse scenes at fine voxel sizes, C5):
// instead of one global hash table hit by two random memory-side atomics per
// point, the points are binned by a hash of their voxel into kHBins bins (the
// brick path's count / scan / scatter shape: one LDS histogram per block,
// runs written contiguously), then one workgroup per bin takes the max index
// per distinct voxel in an LDS hash table.  Every voxel lands in exactly one
// bin, so the per-bin maxima are the global ones.
// The hash is a bijection of the k-bit linear voxel id (xorshifts and odd
// multiplies mod 2^k), so a voxel is its bin (top 12 bits) plus the other
// k - 12 bits: one 8-B entry (rest << 32 | point index) per point, a 4-B LDS
// key.  A bin whose distinct voxels fill its LDS table, or points outside the
// grid, set err bits 4 / 8 and the caller redoes the call with the global
// hash table.
constexpr int kHBins = 4096;                  // = kMaxBuckets (count histogram in LDS)
constexpr int kHBinBits = 12;
constexpr int kHSlotsMax = 16384;             // LDS table per bin: 16384 x (4 B key + 4 B max)
constexpr int kHReduceBlock = 1024;
constexpr int kHMaxBits = kHBinBits + 31;     // the rest must fit 31 bits (0xFFFFFFFF = empty)

struct HMix {
  int k;          // bits of the linear voxel id
  int sh;         // xorshift
  uint64_t mask;  // 2^k - 1
};

__device__ __forceinline__ uint64_t hmix(uint64_t h, const HMix& m) {
  h ^= h >> m.sh;
  h = (h * 0x9E3779B97F4A7C15ull) & m.mask;
  h ^= h >> m.sh;
  h = (h * 0xC2B2AE3D27D4EB4Full) & m.mask;
  h ^= h >> m.sh;
  return h;
}

// the point's mixed voxel id, false when the point is outside the grid
__device__ __forceinline__ bool voxel_hid(const P3& q, const VoxelGeom& g, const HMix& m, uint64_t* h) {
  int v[3];
  if (!voxel_of(q, g, v)) return false;
  *h = hmix((uint64_t)v[0] + (uint64_t)g.nx * ((uint64_t)v[1] + (uint64_t)g.ny * (uint64_t)v[2]), m);
  return true;
}

__device__ __forceinline__ int hbin_of(uint64_t h, const HMix& m) { return (int)(h >> (m.k - kHBinBits)); }

// Blocks of the hash-binned passes: each takes a contiguous chunk of `chunk`
// points (a multiple of kBinRound).  At most kHBinBlocks blocks: the
// bin-major histogram (kHBins x blocks ints), its scan and the per-block
// runs scale with the block count, so few large blocks keep the histogram
// small and each (bin, block) run long (C5's 200M points: 12.2K blocks of 16K
// wrote a 200 MB histogram whose scan alone took 1 ms, and runs of ~4
// entries per bin and block).
constexpr int kHBinBlocks = 2048;
static int hbin_grid(int64_t n, int* chunk) {
  const int64_t nb0 = std::min<int64_t>(std::max<int64_t>(1, (n + kBinChunk - 1) / kBinChunk), kHBinBlocks);
  int64_t c = (n + nb0 - 1) / nb0;
  c = (c + kBinRound - 1) / kBinRound * kBinRound;
  *chunk = (int)c;
  return (int)std::max<int64_t>(1, (n + c - 1) / c);
}

__global__ void __launch_bounds__(kBinBlock) k_hbin_count(const float* __restrict__ xyz, int64_t n, VoxelGeom g,
                                                       HMix m, int chunk, int32_t* __restrict__ bhist,
                                                       int* __restrict__ err) {
  __shared__ int32_t hist[kHBins];
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int k = threadIdx.x; k < kHBins; k += kBinBlock) hist[k] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * chunk, end = min(base + chunk, n);
  bool bad = false;
  constexpr int kU = 8;  // loads in flight per thread
  for (int64_t i0 = base + threadIdx.x; i0 < end; i0 += (int64_t)kU * kBinBlock) {
    P3 q[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) q[u] = p[min(i0 + (int64_t)u * kBinBlock, end - 1)];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (i0 + (int64_t)u * kBinBlock >= end) break;
      uint64_t h;
      if (voxel_hid(q[u], g, m, &h))
        atomicAdd(&hist[hbin_of(h, m)], 1);
      else
        bad = true;
    }
  }
  if (bad) *err = 8;
  __syncthreads();
  for (int k = threadIdx.x; k < kHBins; k += kBinBlock) bhist[(int64_t)k * gridDim.x + blockIdx.x] = hist[k];
}

// dynamic LDS: stage[kBinRound] (u64), cur[kHBins], loc[kHBins]
inline size_t hscatter_lds_bytes() { return kBinRound * sizeof(uint64_t) + 2 * (size_t)kHBins * sizeof(int32_t); }

__global__ void __launch_bounds__(kBinBlock) k_hbin_scatter(const float* __restrict__ xyz, int64_t n, VoxelGeom g,
                                                         HMix m, int chunk, const int32_t* __restrict__ boff,
                                                         uint64_t* __restrict__ entries) {
  extern __shared__ uint64_t lds_u64[];
  uint64_t* stage = lds_u64;
  int32_t* cur = reinterpret_cast<int32_t*>(lds_u64 + kBinRound);  // global address of stage slot 0, per bin
  int32_t* loc = cur + kHBins;                                       // round: count -> offset -> cursor
  __shared__ int32_t wsum[kBinBlock / 64 + 1];
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int k = threadIdx.x; k < kHBins; k += kBinBlock) cur[k] = boff[(int64_t)k * gridDim.x + blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * chunk;
  constexpr int kPer = kBinRound / kBinBlock;
  constexpr int span = kHBins / kBinBlock;
  const int rbits = m.k - kHBinBits;
  for (int r0 = 0; r0 < chunk && base + r0 < n; r0 += kBinRound) {
    for (int k = threadIdx.x; k < kHBins; k += kBinBlock) loc[k] = 0;
    __syncthreads();
    // staged entry per point: rest << 24 | bin << 12 | position in the round
    // (~0: none).  The rest takes up to 31 bits, the bin 12 and the round
    // position 12 (kBinRound = 4096), so no field overlaps another for any
    // k <= kHMaxBits; the point index is re-formed from the position on the
    // way out.
    static_assert(kBinRound == 4096 && kHBinBits == 12, "staged entry layout");
    uint64_t en[kPer];
    P3 q[kPer];
    const int64_t lim = min(base + chunk, n);
#pragma unroll
    for (int j = 0; j < kPer; ++j) q[j] = p[min(base + r0 + threadIdx.x + (int64_t)j * kBinBlock, lim - 1)];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int pos = threadIdx.x + j * kBinBlock;
      const int64_t i = base + r0 + pos;
      uint64_t h;
      en[j] = ~0ull;
      if (i < lim && voxel_hid(q[j], g, m, &h)) {
        const int bin = hbin_of(h, m);
        en[j] = ((h & ((1ull << rbits) - 1)) << 24) | ((uint64_t)bin << 12) | (uint64_t)pos;
        atomicAdd(&loc[bin], 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    const int k0 = threadIdx.x * span, k1 = k0 + span;
    int run = 0;
    for (int k = k0; k < k1; ++k) run += loc[k];
    int tot;
    int ex = block_excl_scan<kBinBlock>(run, wsum, &tot);
    for (int k = k0; k < k1; ++k) {
      const int c = loc[k];
      loc[k] = ex;
      cur[k] -= ex;
      ex += c;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (en[j] == ~0ull) continue;
      stage[atomicAdd(&loc[(int)((en[j] >> 12) & 0xfff)], 1)] = en[j];
    }
    __syncthreads();
    // global entry: rest << 32 | point index (the rest < 2^31, so a key never
    // equals the reduce's empty marker 0xFFFFFFFF)
    for (int t = threadIdx.x; t < tot; t += kBinBlock) {
      const uint64_t e = stage[t];
      const uint32_t i = (uint32_t)(base + r0 + (int64_t)(e & 0xfff));
      entries[cur[(int)((e >> 12) & 0xfff)] + t] = ((e >> 24) << 32) | i;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kHBins; k += kBinBlock) cur[k] += loc[k];
    __syncthreads();
  }
}

// One workgroup per bin: the max index per distinct voxel in an LDS hash table
// of `slots` (power of two) entries; flags[rep] = 1; with the trace, rep by
// global slot (bin * slots + slot) and each point's global slot.
__global__ void __launch_bounds__(kHReduceBlock) k_hbin_reduce(const uint64_t* __restrict__ entries,
                                                               const int32_t* __restrict__ boff, int nblk, int slots,
                                                               uint8_t* __restrict__ flags, int32_t* __restrict__ rep,
                                                               int32_t* __restrict__ vid, int* __restrict__ err) {
  __shared__ uint32_t hk[kHSlotsMax];
  __shared__ int32_t hr[kHSlotsMax];
  __shared__ int full;
  for (int k = threadIdx.x; k < slots; k += kHReduceBlock) {
    hk[k] = 0xFFFFFFFFu;
    hr[k] = -1;
  }
  if (threadIdx.x == 0) full = 0;
  __syncthreads();
  const int bk = blockIdx.x;
  const uint32_t mask = (uint32_t)slots - 1u;
  const int32_t e0 = boff[(int64_t)bk * nblk], e1 = boff[(int64_t)(bk + 1) * nblk];
  constexpr int kU = 8;  // entry loads in flight per thread
  for (int32_t e0u = e0 + threadIdx.x; e0u < e1; e0u += kU * kHReduceBlock) {
    uint64_t wv[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) wv[u] = entries[min(e0u + u * kHReduceBlock, e1 - 1)];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (e0u + u * kHReduceBlock >= e1) break;
      const uint64_t w = wv[u];
      const uint32_t key = (uint32_t)(w >> 32);
      const int32_t idx = (int32_t)(uint32_t)w;
      uint32_t s = key & mask;  // the rest is already mixed
      int probes = 0;
      while (true) {
        const uint32_t prev = atomicCAS(&hk[s], 0xFFFFFFFFu, key);
        if (prev == 0xFFFFFFFFu || prev == key) break;
        s = (s + 1) & mask;
        if (++probes == slots) break;
      }
      if (probes == slots) {  // the bin's table is full
        full = 1;
        continue;
      }
      atomicMax(&hr[s], idx);
      if (vid) vid[idx] = bk * slots + (int32_t)s;
    }
  }
  __syncthreads();
  if (full) {
    if (threadIdx.x == 0) atomicOr(err, 4);
    return;
  }
  for (int k = threadIdx.x; k < slots; k += kHReduceBlock) {
    const int32_t r = hr[k];
    if (rep) rep[(int64_t)bk * slots + k] = r;
    if (r >= 0) flags[r] = 1;
  }
}

// LDS slots per bin: room for every point of an average bin at load <= 1/2,
// at least 256 (the trace's rep table, kHBins x slots ints, then fits the
// dense-table region) and at most kHSlotsMax
static int hbin_slots(int64_t n) {
  int s = 256;
  while (s < kHSlotsMax && (int64_t)s < 2 * ((n + kHBins - 1) / kHBins)) s <<= 1;
  return s;
}

static HMix hbin_mix(double nvox) {
  HMix m{};
  int k = kHBinBits + 1;
  while (k < 63 && std::ldexp(1.0, k) < nvox) ++k;
  m.k = k;
  m.sh = std::max(1, (k + 1) / 2);
  m.mask = k >= 64 ? ~0ull : (1ull << k) - 1;
  return m;
}

__global__ void __launch_bounds__(kBlock) k_voxel_mark(const int32_t* __restrict__ rep, int64_t nslots,
                                                       uint8_t* __restrict__ flags) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nslots; v += (int64_t)gridDim.x * blockDim.x) {
    int32_t r = rep[v];
    if (r >= 0) flags[r] = 1;
  }
}

// The representatives' count is read on the device (cnt[0] = m, cnt[1] =
// error flag of the assign pass: nothing is gathered then), so the gathers
// are queued before the host reads m back.
__global__ void __launch_bounds__(kBlock) k_gather_xyz(const float* __restrict__ xyz, const int32_t* __restrict__ idx,
                                                       const int64_t* __restrict__ cnt, float* __restrict__ out) {
  if ((int)(cnt[1] & 0xffffffff) != 0) return;
  const int64_t m = cnt[0];
  const P3* p = reinterpret_cast<const P3*>(xyz);
  P3* o = reinterpret_cast<P3*>(out);
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
    o[j] = p[idx[j]];
}

__global__ void __launch_bounds__(kBlock) k_voxel_trace(const float* __restrict__ xyz, int64_t n, VoxelGeom g,
                                                        const int32_t* __restrict__ vid,
                                                        const int32_t* __restrict__ rep,
                                                        const int32_t* __restrict__ pos,
                                                        int32_t* __restrict__ voxel_of_point,
                                                        int32_t* __restrict__ cubic) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t row = pos[rep[vid[i]]];
    if (voxel_of_point) voxel_of_point[i] = row;
    if (cubic) {
      double r[3];
      int v[3];
      voxel_ref(p[i], g, r, v);
      // Open3D: cid += {1,2,4}[c] when (ref_coord(c) - voxel_index(c)) >= 0.5
      int cid = ((r[0] - v[0]) >= 0.5 ? 1 : 0) + ((r[1] - v[1]) >= 0.5 ? 2 : 0) + ((r[2] - v[2]) >= 0.5 ? 4 : 0);
      atomicMax(&cubic[(int64_t)row * 8 + cid], (int32_t)i);
    }
  }
}

// Kept voxel grid: vox[v] = (x, y, z, output row as int bits) of voxel v's
// representative, w = -1 for an empty voxel (the buffer is 0xFF-filled).
// Thread per representative (its row is j): the gather of rep_xyz plus one
// 16-byte scatter, so the normals later read the reps in voxel order.
__global__ void __launch_bounds__(kBlock) k_gather_vox(const float* __restrict__ xyz, const int32_t* __restrict__ idx,
                                                       const int64_t* __restrict__ cnt, VoxelGeom g,
                                                       float* __restrict__ rep_xyz, float4* __restrict__ vox) {
  if ((int)(cnt[1] & 0xffffffff) != 0) return;
  const int64_t m = cnt[0];
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const P3 q = p[idx[j]];
    if (rep_xyz) reinterpret_cast<P3*>(rep_xyz)[j] = q;
    int v[3];
    voxel_of(q, g, v);  // inside the grid: the dense path accepted every point
    vox[v[0] + (int64_t)g.nx * (v[1] + (int64_t)g.ny * v[2])] = make_float4(q.x, q.y, q.z, __int_as_float((int)j));
  }
}

// Occupied cells of 2^3 voxels (thread per cell, one atomic per block): with
// one rep per occupied voxel, m / occ2 gives the cloud's local dimension, from
// which the normals size their search cell.
__device__ __forceinline__ bool voxel_full(const int32_t* t, int64_t i) { return t[i] >= 0; }
__device__ __forceinline__ bool voxel_full(const float4* t, int64_t i) { return __float_as_int(t[i].w) >= 0; }

template <class T>
__global__ void __launch_bounds__(kBlock) k_voxel_occ2(const T* __restrict__ table, VoxelGeom g,
                                                       unsigned long long* __restrict__ occ2) {
  const int cx = (g.nx + 1) / 2, cy = (g.ny + 1) / 2, cz = (g.nz + 1) / 2;
  const int64_t nc = (int64_t)cx * cy * cz;
  unsigned long long c = 0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nc; t += (int64_t)gridDim.x * blockDim.x) {
    const int x0 = (int)(t % cx) * 2, y0 = (int)((t / cx) % cy) * 2, z0 = (int)(t / ((int64_t)cx * cy)) * 2;
    bool any = false;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const int x = x0 + (d & 1), y = y0 + ((d >> 1) & 1), z = z0 + (d >> 2);
      if (x < g.nx && y < g.ny && z < g.nz) any |= voxel_full(table, x + (int64_t)g.nx * (y + (int64_t)g.ny * z));
    }
    c += any;
  }
  __shared__ unsigned long long sh[kBlock / 64];
  c = wave_sum(c);
  if (lane_id() == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += sh[w];
    if (t) atomicAdd(occ2, t);  // one per block: the grid is capped at 1024 blocks
  }
}

static int64_t dense_cap(int64_t n) { return dense_cap_hd(n); }
// binned entries: n for the scanned layout, + 1/2 + 2^20 of segment slack
static int64_t entries_cap(int64_t n) { return entries_cap_hd(n); }
// Path-selection memory (per host thread, never shared): the last geometry
// whose one-pass binning overflowed.  It picks which (equally exact) binning
// path a later call on the same geometry tries first, so that call skips a
// doomed attempt; results never depend on it (every path yields the same reps,
// tests/test_gpu_kernels.py runs each).
static thread_local uint64_t g_fused_overflow_key = ~0ull;
// ... whose copied segments overflowed: the one-pass binning retries with one
// copy per brick (a spatially ordered cloud sends each brick's
// points from a few consecutive blocks, i.e. into one or two copies)
static thread_local uint64_t g_fused_one_copy_key = ~0ull;
static int64_t bin_blocks(int64_t n) { return (n + kBinChunk - 1) / kBinChunk; }
static int64_t bin_hist_ints(int64_t n) { return bin_blocks(n) * kMaxBuckets; }
static int64_t hash_cap(int64_t n) {
  int64_t t = 1024;
  while (t < 2 * n) t <<= 1;
  return t;
}

struct VoxelWs {
  uint64_t* entries;           // brick-binned (local, index) pairs
  int32_t* bhist;              // per-block brick counts, brick-major, and their scan
  int32_t* boff;
  int32_t* table;              // dense rep or hash rep
  unsigned long long* keys;    // hash keys
  int32_t* vid;
  uint8_t* flags;
  int32_t* pos;
  int32_t* scan_tmp;
  char* aabb;
  double* mm;
  int64_t* count;  // [0] = m, [1] = err (as int), [2] occupied 2^3 cells
  BinPlan* plan;   // the pre-launched one-pass binning's plan
};

static size_t carve(Arena& ar, int64_t n, VoxelWs* w) {
  int64_t dc = dense_cap(n), hc = hash_cap(n);
  // one region shared by the dense table or the hash (keys + rep)
  size_t table_bytes = std::max<size_t>(dc * sizeof(int32_t), hc * (sizeof(int32_t) + sizeof(uint64_t)));
  char* tb = ar.take<char>(table_bytes);
  w->table = reinterpret_cast<int32_t*>(tb);
  w->keys = tb ? reinterpret_cast<unsigned long long*>(tb + Arena::align(hc * sizeof(int32_t))) : nullptr;
  w->entries = ar.take<uint64_t>(entries_cap(n));
  w->bhist = ar.take<int32_t>(bin_hist_ints(n));
  w->boff = ar.take<int32_t>(std::max<int64_t>(bin_hist_ints(n) + 1, kTotWords + (int64_t)kMaxBuckets + 1));
  w->vid = ar.take<int32_t>(n);
  w->flags = ar.take<uint8_t>(n + 16);
  w->pos = ar.take<int32_t>(n);
  w->scan_tmp = ar.take<int32_t>(std::max<size_t>(compact_workspace_ints(n), scan_workspace_ints(bin_hist_ints(n) + 1)));
  w->aabb = ar.take<char>(aabb_ws_bytes(n));
  w->mm = ar.take<double>(8);
  w->count = ar.take<int64_t>(8);
  w->plan = ar.take<BinPlan>(1);
  return ar.used;
}

}  // namespace o3dx

using namespace o3dx;

extern "C" size_t o3dx_voxel_workspace_bytes(int64_t n) {
  Arena ar(nullptr, 0);
  VoxelWs w;
  // hash keys live after an aligned rep block inside the table region
  return carve(ar, std::max<int64_t>(n, 1), &w) + Arena::align(hash_cap(std::max<int64_t>(n, 1)) * 4) + 1024;
}

static void voxel_dims(const double mn[3], const double mx[3], double vs, double dims[3]) {
  for (int a = 0; a < 3; ++a) dims[a] = std::floor(std::max(0.0, mx[a] - mn[a]) / vs) + 1.0;
}

extern "C" int64_t o3dx_voxel_grid_capacity(int64_t n) { return n > 0 ? dense_cap(n) : 0; }

extern "C" int64_t o3dx_voxel_grid_cells(int64_t n, const double* min_bound_host, const double* max_bound_host,
                                         double voxel_size) {
  if (!min_bound_host || !max_bound_host || !(voxel_size > 0.0) || n <= 0) return 0;
  double dims[3];
  voxel_dims(min_bound_host, max_bound_host, voxel_size, dims);
  const double nvox = dims[0] * dims[1] * dims[2];
  if (!(nvox <= (double)dense_cap(n))) return 0;
  if (plan_bricks((int)dims[0], (int)dims[1], (int)dims[2]).nb == 0) return 0;
  return (int64_t)nvox;
}

static int voxel_impl(const float* xyz, int64_t n, const double* min_bound_host, const double* max_bound_host,
                      double voxel_size, int32_t* rep_idx, float* rep_xyz, int64_t* m_host, int32_t* voxel_of_point,
                      int32_t* cubic_id, float* vox, int64_t vox_cap, double* geom, void* ws, size_t ws_bytes,
                      void* stream, const int64_t* xwin = nullptr, VoxelHook hook = nullptr, void* hook_ctx = nullptr,
                      ZeroSpan extra_zero = {}, int64_t* counts_dev = nullptr) {
  if (geom)
    for (int k = 0; k < 12; ++k) geom[k] = 0.0;
  if (n < 0 || (n > 0 && (!xyz || !rep_idx)) || !m_host)
    return fail(O3DX_EINVAL, "o3dx_voxel_down_sample: bad arguments");
  if (!(voxel_size > 0.0)) return fail(O3DX_EINVAL, "voxel_size <= 0.");
  if (ws_bytes < o3dx_voxel_workspace_bytes(n) || !ws)
    return fail(O3DX_ENOMEM, "o3dx_voxel_down_sample: workspace too small (need %zu)", o3dx_voxel_workspace_bytes(n));
  hipStream_t s = as_stream(stream);
  Arena ar(ws, ws_bytes);
  VoxelWs w;
  carve(ar, std::max<int64_t>(n, 1), &w);
  w.keys = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w.table) +
                                                 Arena::align(hash_cap(std::max<int64_t>(n, 1)) * 4));

  double mn[3], mx[3];
  // the clears that do not depend on the geometry run while the host waits
  // for the bounds (the first attempt below skips them)
  auto clears = [&]() -> int {
    O3DX_HIP(hipMemsetAsync(w.count, 0, 8 * sizeof(int64_t), s));
    O3DX_HIP(hipMemsetAsync(w.boff, 0, (size_t)kTotWords * sizeof(int32_t), s));
    if (n > 0) O3DX_HIP(hipMemsetAsync(w.flags, 0, n, s));
    return 0;
  };
  // one-pass binning allowed (the plan decides whether it applies)
  // O3DX_VOXEL_TWOPASS (tests): the count + scatter path, the one-pass binning's fall-back
  const int allow_fused = !getenv("O3DX_VOXEL_TWOPASS") ? 1 : 0;
  bool pre_launched = false;
  if (!min_bound_host || !max_bound_host) {
    double mm[6];
    const ZeroSpan zc{reinterpret_cast<uint8_t*>(w.count), 8 * sizeof(int64_t)};
    const ZeroSpan zb{reinterpret_cast<uint8_t*>(w.boff), (size_t)kTotWords * sizeof(int32_t)};
    const ZeroSpan zf{w.flags, (size_t)n};
    if (!min_bound_host && !max_bound_host && allow_fused && n > 0) {
      // the bounds' final kernel also forms the one-pass binning's plan,
      // and the binning starts on it while the host waits for the bounds (the
      // host replays the same plan below)
      AabbOut o;
      const float* part;
      int nb;
      O3DX_TRY(aabb_begin_partial(xyz, n, w.aabb, s, zc, zb, zf, extra_zero, &o, &part, &nb));
      const PlanTail tail{voxel_size, n, allow_fused, g_fused_overflow_key, g_fused_one_copy_key, w.plan};
      hipLaunchKernelGGL(k_aabb_final_tail<PlanTail>, dim3(1), dim3(kBlock), 0, s, part, nb, n, o, tail);
      launch_fused<true>(kFuseMaxBricks, n, s, xyz, n, (const BinPlan*)w.plan, w.boff, w.entries,
                         (voxel_of_point || cubic_id) ? w.vid : nullptr, reinterpret_cast<int*>(w.count + 1));
      pre_launched = true;
    } else {
      O3DX_TRY(aabb_begin(xyz, n, w.aabb, s, zc, zb, zf, extra_zero));
    }
    O3DX_TRY(aabb_end(mm, s));
    for (int a = 0; a < 3; ++a) {
      mn[a] = min_bound_host ? min_bound_host[a] : mm[a];
      mx[a] = max_bound_host ? max_bound_host[a] : mm[3 + a];
    }
  } else {
    O3DX_TRY(clears());
    for (int a = 0; a < 3; ++a) {
      mn[a] = min_bound_host[a];
      mx[a] = max_bound_host[a];
    }
  }
  // Open3D: if (voxel_size * INT_MAX < (max_bound - min_bound).maxCoeff()) LogError
  double ext = std::max(mx[0] - mn[0], std::max(mx[1] - mn[1], mx[2] - mn[2]));
  if (voxel_size * (double)INT32_MAX < ext) return fail(O3DX_EINVAL, "voxel_size is too small.");
  if (n == 0) {
    *m_host = 0;
    return 0;
  }
  VoxelGeom g;
  g.mnx = mn[0];
  g.mny = mn[1];
  g.mnz = mn[2];
  g.vs = voxel_size;
  g.ivs = 1.0 / voxel_size;
  double dims[3];
  voxel_dims(mn, mx, voxel_size, dims);
  if (xwin) {  // slab: only the x keys [xwin[0], xwin[1]) exist, every point must fall inside
    if (xwin[0] < 0 || xwin[1] <= xwin[0] || (double)xwin[1] > dims[0])
      return fail(O3DX_EINVAL, "o3dx_voxel_down_sample_window: bad x-key window");
    g.kx0 = (int)xwin[0];
    dims[0] = (double)(xwin[1] - xwin[0]);
  }
  double nvox = dims[0] * dims[1] * dims[2];
  bool dense = nvox <= (double)dense_cap(n);
  if (xwin && !dense) return fail(O3DX_ENOTSUP, "o3dx_voxel_down_sample_window: slab grid too sparse for a table");
  g.nx = (int)dims[0];
  g.ny = (int)dims[1];
  g.nz = (int)dims[2];

  const unsigned grid = grid_for(n, kBlock, 8192);
  int64_t counts[3];
  bool grid_kept = false;
  // sparse grids: hash-binned reduction from kHBinMin points (below it the
  // global table is small enough to stay in cache), the global hash table
  // otherwise or when a bin's LDS table overflowed
  int64_t hbin_min = (int64_t)1 << 22;
  if (const char* e = getenv("O3DX_VOXEL_HBIN_MIN")) hbin_min = atoll(e);  // tests / tuning
  bool hbin_ok = hbin_min >= 0;
  bool fused_ok = true;
  int attempts_made = 0;
  HostPost counts_post;
  int fused_ncp = 0;  // segment copies of the attempt's one-pass binning (0: not that path)
  for (int attempt = 0; attempt < 5; ++attempt) {
    fused_ncp = 0;
    attempts_made = attempt;
    bool posted = false;
    grid_kept = false;
    int64_t nslots;
    if (attempt > 0) O3DX_TRY(clears());
    Bricks bricks = dense ? plan_bricks(g.nx, g.ny, g.nz) : Bricks{};
    if (dense && bricks.nb > 0) {
      nslots = (int64_t)nvox;
      const unsigned nblk = (unsigned)((n + kBinChunk - 1) / kBinChunk);
      KTimer kt("voxel_assign", s);
      // the brick totals (w.boff, cleared with the counts)
      int32_t* btot = w.boff;
      int32_t* bbase = w.boff + (size_t)kTotWords;
      // one pass into fixed per-brick segments when a segment holds a full
      // brick's share of a uniform cloud with room to spare (and this
      // geometry did not overflow last time)
      BinPlan plan;
      if (xwin)  // the slab's window: its own geometry (round 4; count + scatter before)
        fused_plan_geom(g, n, fused_ok && allow_fused, g_fused_overflow_key, &plan, g_fused_one_copy_key);
      else
        fused_plan(mn, mx, voxel_size, n, fused_ok && allow_fused, g_fused_overflow_key, &plan, g_fused_one_copy_key);
      const bool fused = plan.ok;
      fused_ncp = fused ? plan.b.ncp : 0;
      if (fused) bricks = plan.b;  // the one-pass plan's (larger) bricks
      const int cap = fused ? plan.cap : 0;
      if (fused && attempt == 0 && pre_launched) {
        // already running on the device's identical plan
      } else if (fused) {
        launch_fused<false>(bricks.nb, n, s, xyz, n, g, bricks, cap, btot, w.entries,
                     (voxel_of_point || cubic_id) ? w.vid : nullptr, reinterpret_cast<int*>(w.count + 1));
      } else {
        hipLaunchKernelGGL(k_vbin_count, dim3(nblk), dim3(kBinBlock), 0, s, xyz, n, g, bricks, w.bhist, btot,
                           (voxel_of_point || cubic_id) ? w.vid : nullptr, reinterpret_cast<int*>(w.count + 1));
        hipLaunchKernelGGL(k_vbin_scatter, dim3(nblk), dim3(kBinBlock), scatter_lds_bytes(bricks.nb), s, xyz, n, g,
                           bricks, w.bhist, btot, bbase, w.entries);
      }
      const bool keep = vox && nslots <= vox_cap;
      const bool occ_in_reduce = keep && bricks.sx >= 1 && bricks.sy >= 1 && bricks.sz >= 1;
      const bool trace = voxel_of_point || cubic_id;
      // the int32 table is only read by the trace and the standalone occupancy pass
      hipLaunchKernelGGL(k_vbin_reduce, dim3(bricks.nb), dim3(kReduceBlock), 0, s, w.entries, bbase, cap, btot, g,
                         bricks,
                         (trace || (keep && !occ_in_reduce)) ? w.table : nullptr, w.flags,
                         occ_in_reduce ? reinterpret_cast<unsigned long long*>(w.count + 2) : nullptr,
                         keep ? reinterpret_cast<float4*>(vox) : nullptr);
      kt.stop();
      KTimer kc("voxel_compact", s);
      if (keep) {
        if (!occ_in_reduce) {
          const int64_t nc2 = (int64_t)((g.nx + 1) / 2) * ((g.ny + 1) / 2) * ((g.nz + 1) / 2);
          hipLaunchKernelGGL(k_voxel_occ2<int32_t>, dim3(grid_for(nc2, kBlock, 1024)), dim3(kBlock), 0, s, w.table,
                             g, reinterpret_cast<unsigned long long*>(w.count + 2));
        }
        grid_kept = true;
      }
      // (measured: a compaction fused with an in-order gather of the reps'
      // xyz + a thread-per-rep table fill took 54 + 36 us against 14 + 56 us
      // for the compaction + k_gather_vox below at C2 — the sparse in-order
      // read of the cloud costs what the random gather does)
      // the one-call pipeline (a hook, attempt 0): the counts go to the host
      // from the compaction's last kernel, not by a copy queued after the gathers
      if (hook && keep && attempt == 0) {
        O3DX_TRY(post_prepare(&counts_post));
        posted = true;
      }
      O3DX_TRY(compact_flags(w.flags, n, rep_idx, (voxel_of_point || cubic_id) ? w.pos : nullptr, w.count,
                             w.scan_tmp, s, posted ? &counts_post : nullptr, 3));
    } else if (!dense && hbin_ok && n >= hbin_min && hbin_mix(nvox).k <= kHMaxBits) {
      int hchunk;
      const unsigned nblk = (unsigned)hbin_grid(n, &hchunk);
      const HMix hm = hbin_mix(nvox);
      int slots = hbin_slots(n);
      if (const char* e = getenv("O3DX_VOXEL_HBIN_SLOTS"))  // tests: force the overflow fall-back
        slots = std::max(2, std::min(slots, atoi(e)));
      const bool trace = voxel_of_point || cubic_id;
      KTimer kt("voxel_assign", s);
      hipLaunchKernelGGL(k_hbin_count, dim3(nblk), dim3(kBinBlock), 0, s, xyz, n, g, hm, hchunk, w.bhist,
                         reinterpret_cast<int*>(w.count + 1));
      O3DX_TRY(exclusive_scan_i32(w.bhist, w.boff, (int64_t)kHBins * nblk, w.scan_tmp, s));
      hipLaunchKernelGGL(k_hbin_scatter, dim3(nblk), dim3(kBinBlock), hscatter_lds_bytes(), s, xyz, n, g, hm, hchunk, w.boff,
                         w.entries);
      hipLaunchKernelGGL(k_hbin_reduce, dim3(kHBins), dim3(kHReduceBlock), 0, s, w.entries, w.boff, (int)nblk, slots,
                         w.flags, trace ? w.table : nullptr, trace ? w.vid : nullptr,
                         reinterpret_cast<int*>(w.count + 1));
      kt.stop();
      KTimer kc("voxel_compact", s);
      O3DX_TRY(compact_flags(w.flags, n, rep_idx, trace ? w.pos : nullptr, w.count, w.scan_tmp, s));
    } else {
      if (dense) {
        nslots = (int64_t)nvox;
        O3DX_HIP(hipMemsetAsync(w.table, 0xFF, nslots * sizeof(int32_t), s));
        KTimer kt("voxel_assign", s);
        hipLaunchKernelGGL(k_voxel_assign_dense, dim3(grid), dim3(kBlock), 0, s, xyz, n, g, w.table, w.vid,
                           reinterpret_cast<int*>(w.count + 1));
        hipLaunchKernelGGL(k_voxel_settle, dim3(grid), dim3(kBlock), 0, s, w.vid, n, w.table);
      } else {
        nslots = hash_cap(n);
        O3DX_HIP(hipMemsetAsync(w.table, 0xFF, nslots * sizeof(int32_t), s));
        O3DX_HIP(hipMemsetAsync(w.keys, 0xFF, nslots * sizeof(uint64_t), s));
        KTimer kt("voxel_assign", s);
        hipLaunchKernelGGL(k_voxel_assign_hash, dim3(grid), dim3(kBlock), 0, s, xyz, n, g, w.keys, w.table,
                           (uint32_t)(nslots - 1), w.vid, reinterpret_cast<int*>(w.count + 1));
      }
      KTimer kt("voxel_compact", s);
      hipLaunchKernelGGL(k_voxel_mark, dim3(grid_for(nslots, kBlock, 8192)), dim3(kBlock), 0, s, w.table, nslots,
                         w.flags);
      O3DX_TRY(compact_flags(w.flags, n, rep_idx, (voxel_of_point || cubic_id) ? w.pos : nullptr, w.count,
                             w.scan_tmp, s));
    }
    const bool early = hook && grid_kept && attempt == 0;
    // gathers sized by the device-side count (at most n rows), queued ahead
    // of the read-back so they overlap the host round trip
    const unsigned gg = grid_for(n, kBlock, 8192);
    if (grid_kept)
      hipLaunchKernelGGL(k_gather_vox, dim3(gg), dim3(kBlock), 0, s, xyz, rep_idx, w.count, g, rep_xyz,
                         reinterpret_cast<float4*>(vox));
    else if (rep_xyz)
      hipLaunchKernelGGL(k_gather_xyz, dim3(gg), dim3(kBlock), 0, s, xyz, rep_idx, w.count, rep_xyz);
    if (counts_dev) {
      // deferred (o3dx_voxel_down_sample_window_deferred): {m, error bits,
      // occupancy} stay on the device for the caller; no retry (an overflow
      // of the one-pass binning is error bit 16, the caller re-runs the
      // synchronous form)
      O3DX_HIP(hipMemcpyAsync(counts_dev, w.count, 3 * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
      O3DX_HIP(hipGetLastError());
      *m_host = -1;
      return 0;
    }
    if (early) {
      // the hook's work (the table geometry, occupancy not yet known) is
      // queued right behind the gathers; the host then waits for the counts
      // the compaction posted (earlier: a 5 us copy kernel queued in between)
      const double gv[12] = {g.mnx + (double)g.kx0 * g.vs, g.mny, g.mnz, g.vs, (double)g.nx, (double)g.ny,
                             (double)g.nz, 1.0, -1.0, (double)g.kx0, 0.0, nvox};
      O3DX_TRY(hook(hook_ctx, gv, vox));
      if (posted)
        O3DX_TRY(post_wait(counts_post, counts, 3 * sizeof(int64_t), s));
      else
        O3DX_TRY(read_back(counts, w.count, 3 * sizeof(int64_t), s));
    } else {
      O3DX_TRY(read_back(counts, w.count, 3 * sizeof(int64_t), s));
    }
    int errflag = (int)(counts[1] & 0xffffffff);
    if (errflag == 0) break;
    if (errflag & 16) {  // a brick outgrew its one-pass segment (remembered per geometry):
      if (fused_ncp > 1) {  // copied segments: one copy per brick next
        g_fused_one_copy_key = geom_key(g, n);
      } else {  // one copy: count + scatter
        g_fused_overflow_key = geom_key(g, n);
        fused_ok = false;
      }
      if (!(errflag & ~16)) continue;
      errflag &= ~16;
    }
    if ((errflag & 12) && !(errflag & ~12)) {  // hash-binned path: bin table full / point outside: global hash
      hbin_ok = false;
      continue;
    }
    if (xwin) return fail(O3DX_EINVAL, "o3dx_voxel_down_sample_window: points outside the x-key window");
    if (errflag == 2 || !dense)
      return fail(O3DX_ENOTSUP, "voxel grid spans more than 2^%d cells per axis", kHashBits);
    dense = false;  // points outside the given bounds: retry with the hash table
  }
  const int64_t m = counts[0];
  *m_host = m;
  if (geom && grid_kept) {
    // geom[10]: the attempt that built the table (> 0: a hook fired on attempt
    // 0 saw a table that was rebuilt since)
    const double gv[12] = {g.mnx + (double)g.kx0 * g.vs, g.mny, g.mnz, g.vs, (double)g.nx, (double)g.ny,
                           (double)g.nz, 1.0, (double)counts[2], (double)g.kx0, (double)attempts_made, nvox};
    for (int k = 0; k < 12; ++k) geom[k] = gv[k];
  }
  if ((voxel_of_point || cubic_id) && m > 0) {
    if (cubic_id) O3DX_HIP(hipMemsetAsync(cubic_id, 0xFF, (size_t)m * 8 * sizeof(int32_t), s));
    hipLaunchKernelGGL(k_voxel_trace, dim3(grid), dim3(kBlock), 0, s, xyz, n, g, w.vid, w.table, w.pos,
                       voxel_of_point, cubic_id);
  }
  O3DX_HIP(hipGetLastError());
  return 0;
}

extern "C" int o3dx_voxel_down_sample(const float* xyz, int64_t n, const double* min_bound_host,
                                      const double* max_bound_host, double voxel_size, int32_t* rep_idx,
                                      float* rep_xyz, int64_t* m_host, int32_t* voxel_of_point, int32_t* cubic_id,
                                      void* ws, size_t ws_bytes, void* stream) {
  return voxel_impl(xyz, n, min_bound_host, max_bound_host, voxel_size, rep_idx, rep_xyz, m_host, voxel_of_point,
                    cubic_id, nullptr, 0, nullptr, ws, ws_bytes, stream);
}

extern "C" int o3dx_voxel_down_sample_grid(const float* xyz, int64_t n, const double* min_bound_host,
                                           const double* max_bound_host, double voxel_size, int32_t* rep_idx,
                                           float* rep_xyz, int64_t* m_host, int32_t* voxel_of_point,
                                           int32_t* cubic_id, float* voxel_pts, int64_t voxel_cells,
                                           double* geom_host, void* ws, size_t ws_bytes, void* stream) {
  if (!voxel_pts || !geom_host) return fail(O3DX_EINVAL, "o3dx_voxel_down_sample_grid: null voxel_pts / geom");
  return voxel_impl(xyz, n, min_bound_host, max_bound_host, voxel_size, rep_idx, rep_xyz, m_host, voxel_of_point,
                    cubic_id, voxel_pts, voxel_cells, geom_host, ws, ws_bytes, stream);
}

extern "C" int o3dx_voxel_down_sample_window(const float* xyz, int64_t n, const double* min_bound_host,
                                             const double* max_bound_host, double voxel_size, int64_t kx0,
                                             int64_t kx1, int32_t* rep_idx, float* rep_xyz, int64_t* m_host,
                                             float* voxel_pts, int64_t voxel_cells, double* geom_host, void* ws,
                                             size_t ws_bytes, void* stream) {
  if (!min_bound_host || !max_bound_host)
    return fail(O3DX_EINVAL, "o3dx_voxel_down_sample_window: the global bounds are required");
  const int64_t win[2] = {kx0, kx1};
  return voxel_impl(xyz, n, min_bound_host, max_bound_host, voxel_size, rep_idx, rep_xyz, m_host, nullptr, nullptr,
                    voxel_pts, voxel_pts ? voxel_cells : 0, geom_host, ws, ws_bytes, stream, win);
}

extern "C" int o3dx_voxel_down_sample_window_deferred(const float* xyz, int64_t n, const double* min_bound_host,
                                                      const double* max_bound_host, double voxel_size, int64_t kx0,
                                                      int64_t kx1, int32_t* rep_idx, float* rep_xyz,
                                                      int64_t* counts_dev, void* ws, size_t ws_bytes, void* stream) {
  if (!min_bound_host || !max_bound_host || !counts_dev)
    return fail(O3DX_EINVAL, "o3dx_voxel_down_sample_window_deferred: bounds and counts_dev are required");
  const int64_t win[2] = {kx0, kx1};
  int64_t m_host = 0;
  if (n == 0) {  // nothing queued: the counts are zero
    O3DX_HIP(hipMemsetAsync(counts_dev, 0, 3 * sizeof(int64_t), as_stream(stream)));
  }
  return voxel_impl(xyz, n, min_bound_host, max_bound_host, voxel_size, rep_idx, rep_xyz, &m_host, nullptr, nullptr,
                    nullptr, 0, nullptr, ws, ws_bytes, stream, win, nullptr, nullptr, {}, counts_dev);
}

// ------------------------------------------------------ float64 clouds
// The float64 boundary (include/o3dx.h): Open3D computes the voxel key of
// its float64 points, ref = (p - min_bound) / voxel_size, key = int(floor(ref)),
// octant bit (ref - key) >= 0.5 (PointCloud::VoxelDownSampleAndTrace;
// reference PointCloud.py:338-341 on float64 storage, :99-102).  The keys
// kernel evaluates exactly that in float64 and encodes key + 0.25 (octant bit
// clear) or key + 0.75 (set) as a float32 coordinate — exact for |key| <
// 2^22 — so the integer pipeline above runs unchanged on (min 0, voxel size
// 1): floor(key + 0.25 / 0.75) is the key, the fraction the octant bit, and
// every representative (max index per voxel), trace row and octant id is the
// float64 computation's.
constexpr double kKey64Lim = 4194304.0;  // 2^22

__global__ void __launch_bounds__(kBlock) k_voxel_keys64(const double* __restrict__ xyz, int64_t n, double mnx,
                                                         double mny, double mnz, double vs, float* __restrict__ out,
                                                         int* __restrict__ err) {
  const double mn[3] = {mnx, mny, mnz};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const double r = (xyz[3 * i + a] - mn[a]) / vs;
      const double k = floor(r);
      if (!(fabs(k) < kKey64Lim)) *err = 1;  // NaN too
      out[3 * i + a] = (float)(k + ((r - k) >= 0.5 ? 0.75 : 0.25));
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_gather_xyz64(const double* __restrict__ xyz, const int32_t* __restrict__ idx,
                                                         int64_t m, double* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx[j];
    out[3 * j] = xyz[3 * i];
    out[3 * j + 1] = xyz[3 * i + 1];
    out[3 * j + 2] = xyz[3 * i + 2];
  }
}

extern "C" size_t o3dx_voxel_f64_workspace_bytes(int64_t n) {
  n = std::max<int64_t>(n, 1);
  return o3dx_voxel_workspace_bytes(n) + Arena::align((size_t)n * 3 * sizeof(float) + 1) +
         Arena::align(aabb64_ws_bytes() + 64) + 1024;
}

extern "C" int o3dx_voxel_down_sample_f64(const double* xyz, int64_t n, const double* min_bound_host,
                                          const double* max_bound_host, double voxel_size, int32_t* rep_idx,
                                          double* rep_xyz, int64_t* m_host, int32_t* voxel_of_point,
                                          int32_t* cubic_id, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !rep_idx)) || !m_host)
    return fail(O3DX_EINVAL, "o3dx_voxel_down_sample_f64: bad arguments");
  if (!(voxel_size > 0.0)) return fail(O3DX_EINVAL, "voxel_size <= 0.");
  if (!ws || ws_bytes < o3dx_voxel_f64_workspace_bytes(n))
    return fail(O3DX_ENOMEM, "o3dx_voxel_down_sample_f64: workspace too small (need %zu)",
                o3dx_voxel_f64_workspace_bytes(n));
  hipStream_t s = as_stream(stream);
  Arena ar(ws, ws_bytes);
  float* keys = ar.take<float>((size_t)std::max<int64_t>(n, 1) * 3);
  char* aws = ar.take<char>(aabb64_ws_bytes() + 64);
  const size_t vbytes = o3dx_voxel_workspace_bytes(n);
  char* vws = ar.take<char>(vbytes);
  O3DX_ARENA_CHECK(ar);
  double mn[3], mx[3];
  double* mmd = reinterpret_cast<double*>(aws + aabb64_ws_bytes());
  if (!min_bound_host || !max_bound_host) {
    double mm[6];
    O3DX_TRY(aabb64_device(xyz, n, mmd, aws, s));
    O3DX_TRY(read_back(mm, mmd, sizeof(mm), s));
    for (int a = 0; a < 3; ++a) {
      mn[a] = min_bound_host ? min_bound_host[a] : mm[a];
      mx[a] = max_bound_host ? max_bound_host[a] : mm[3 + a];
    }
  } else {
    for (int a = 0; a < 3; ++a) {
      mn[a] = min_bound_host[a];
      mx[a] = max_bound_host[a];
    }
  }
  const double ext = std::max(mx[0] - mn[0], std::max(mx[1] - mn[1], mx[2] - mn[2]));
  if (voxel_size * (double)INT32_MAX < ext) return fail(O3DX_EINVAL, "voxel_size is too small.");
  if (n == 0) {
    *m_host = 0;
    return 0;
  }
  double dims[3];
  voxel_dims(mn, mx, voxel_size, dims);
  for (int a = 0; a < 3; ++a)
    if (!(dims[a] <= kKey64Lim)) return fail(O3DX_ENOTSUP, "voxel grid spans more than 2^22 cells per axis");
  int* err = reinterpret_cast<int*>(mmd + 6);
  O3DX_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_voxel_keys64, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, mn[0], mn[1], mn[2],
                     voxel_size, keys, err);
  if (min_bound_host && max_bound_host) {  // points outside caller bounds may leave the exact key range
    int e = 0;
    O3DX_TRY(read_back(&e, err, sizeof(int), s));
    if (e) return fail(O3DX_ENOTSUP, "voxel keys beyond 2^22 cells (points far outside the bounds?)");
  }
  const double kmn[3] = {0.0, 0.0, 0.0}, kmx[3] = {dims[0] - 0.5, dims[1] - 0.5, dims[2] - 0.5};
  O3DX_TRY(voxel_impl(keys, n, kmn, kmx, 1.0, rep_idx, nullptr, m_host, voxel_of_point, cubic_id, nullptr, 0,
                      nullptr, vws, vbytes, stream));
  const int64_t m = *m_host;
  if (rep_xyz && m > 0)
    hipLaunchKernelGGL(k_gather_xyz64, dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, xyz, rep_idx, m, rep_xyz);
  O3DX_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------ table build
// The voxel table of an arbitrary point set holding at most one point per
// voxel (a slab's own + halo representatives): vox[v] = (x, y, z, row).
// skip_nonfinite: rows with a non-finite coordinate are padding (the deferred
// form); err: int bits (the read-back form) or, with err64, int64 bits.
__global__ void __launch_bounds__(kBlock) k_table_build(const float* __restrict__ xyz, int64_t n, VoxelGeom g,
                                                        float4* __restrict__ vox, int* __restrict__ err,
                                                        unsigned long long* __restrict__ err64 = nullptr,
                                                        int skip_nonfinite = 0) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const P3 q = p[j];
    if (skip_nonfinite && !(__builtin_isfinite(q.x) && __builtin_isfinite(q.y) && __builtin_isfinite(q.z))) continue;
    int v[3];
    if (!voxel_of(q, g, v)) {
      if (err64) atomicOr(err64, 1ull);
      else atomicOr(err, 1);
      continue;
    }
    const int64_t at = v[0] + (int64_t)g.nx * (v[1] + (int64_t)g.ny * v[2]);
    int* w = reinterpret_cast<int*>(&vox[at].w);
    if (atomicCAS(w, -1, (int)j) != -1) {
      if (err64) atomicOr(err64, 2ull);
      else atomicOr(err, 2);
      continue;
    }
    vox[at].x = q.x;
    vox[at].y = q.y;
    vox[at].z = q.z;
  }
}

extern "C" size_t o3dx_voxel_table_workspace_bytes(void) { return 256; }

extern "C" int o3dx_voxel_table_build(const float* xyz, int64_t n, const double* min_bound_host,
                                      const double* max_bound_host, double voxel_size, int64_t kx0, int64_t kx1,
                                      float* voxel_pts, int64_t voxel_cells, double* geom_host, void* ws,
                                      size_t ws_bytes, void* stream) {
  if (geom_host)
    for (int k = 0; k < 12; ++k) geom_host[k] = 0.0;
  if (n < 0 || (n > 0 && !xyz) || !voxel_pts || !geom_host || !min_bound_host || !max_bound_host || !ws ||
      ws_bytes < o3dx_voxel_table_workspace_bytes())
    return fail(O3DX_EINVAL, "o3dx_voxel_table_build: bad arguments");
  if (!(voxel_size > 0.0)) return fail(O3DX_EINVAL, "voxel_size <= 0.");
  double dims[3];
  voxel_dims(min_bound_host, max_bound_host, voxel_size, dims);
  if (kx0 < 0 || kx1 <= kx0 || (double)kx1 > dims[0]) return fail(O3DX_EINVAL, "o3dx_voxel_table_build: bad window");
  VoxelGeom g;
  g.mnx = min_bound_host[0];
  g.mny = min_bound_host[1];
  g.mnz = min_bound_host[2];
  g.vs = voxel_size;
  g.ivs = 1.0 / voxel_size;
  g.kx0 = (int)kx0;
  g.nx = (int)(kx1 - kx0);
  g.ny = (int)dims[1];
  g.nz = (int)dims[2];
  const int64_t nvox = (int64_t)g.nx * g.ny * g.nz;
  if (nvox > voxel_cells) return fail(O3DX_ENOMEM, "o3dx_voxel_table_build: table needs %lld voxels", (long long)nvox);
  hipStream_t s = as_stream(stream);
  int64_t* cnt = reinterpret_cast<int64_t*>(ws);  // [0] error bits, [1] occupied 2^3 cells
  O3DX_HIP(hipMemsetAsync(cnt, 0, 2 * sizeof(int64_t), s));
  O3DX_HIP(hipMemsetAsync(voxel_pts, 0xFF, (size_t)nvox * 4 * sizeof(float), s));
  if (n > 0)
    hipLaunchKernelGGL(k_table_build, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, g,
                       reinterpret_cast<float4*>(voxel_pts), reinterpret_cast<int*>(cnt));
  const int64_t nc2 = (int64_t)((g.nx + 1) / 2) * ((g.ny + 1) / 2) * ((g.nz + 1) / 2);
  hipLaunchKernelGGL(k_voxel_occ2<float4>, dim3(grid_for(nc2, kBlock, 1024)), dim3(kBlock), 0, s,
                     reinterpret_cast<const float4*>(voxel_pts), g, reinterpret_cast<unsigned long long*>(cnt + 1));
  O3DX_HIP(hipGetLastError());
  int64_t c[2];
  O3DX_TRY(read_back(c, cnt, sizeof(c), s));
  if (c[0] & 1) return fail(O3DX_EINVAL, "o3dx_voxel_table_build: points outside the window");
  if (c[0] & 2) return fail(O3DX_EINVAL, "o3dx_voxel_table_build: two points in one voxel");
  const double gv[12] = {g.mnx + (double)g.kx0 * g.vs, g.mny, g.mnz, g.vs, (double)g.nx, (double)g.ny, (double)g.nz,
                         1.0, (double)c[1], (double)g.kx0, 0.0, (double)nvox};
  for (int k = 0; k < 12; ++k) geom_host[k] = gv[k];
  return 0;
}

extern "C" int o3dx_voxel_table_build_deferred(const float* xyz, int64_t n, const double* min_bound_host,
                                               const double* max_bound_host, double voxel_size, int64_t kx0,
                                               int64_t kx1, float* voxel_pts, int64_t voxel_cells, double* geom_host,
                                               int64_t* status_dev, void* stream) {
  if (geom_host)
    for (int k = 0; k < 12; ++k) geom_host[k] = 0.0;
  if (n < 0 || (n > 0 && !xyz) || !voxel_pts || !geom_host || !min_bound_host || !max_bound_host || !status_dev)
    return fail(O3DX_EINVAL, "o3dx_voxel_table_build_deferred: bad arguments");
  if (!(voxel_size > 0.0)) return fail(O3DX_EINVAL, "voxel_size <= 0.");
  double dims[3];
  voxel_dims(min_bound_host, max_bound_host, voxel_size, dims);
  if (kx0 < 0 || kx1 <= kx0 || (double)kx1 > dims[0]) return fail(O3DX_EINVAL, "o3dx_voxel_table_build: bad window");
  VoxelGeom g;
  g.mnx = min_bound_host[0];
  g.mny = min_bound_host[1];
  g.mnz = min_bound_host[2];
  g.vs = voxel_size;
  g.ivs = 1.0 / voxel_size;
  g.kx0 = (int)kx0;
  g.nx = (int)(kx1 - kx0);
  g.ny = (int)dims[1];
  g.nz = (int)dims[2];
  const int64_t nvox = (int64_t)g.nx * g.ny * g.nz;
  if (nvox > voxel_cells) return fail(O3DX_ENOMEM, "o3dx_voxel_table_build: table needs %lld voxels", (long long)nvox);
  hipStream_t s = as_stream(stream);
  O3DX_HIP(hipMemsetAsync(voxel_pts, 0xFF, (size_t)nvox * 4 * sizeof(float), s));
  if (n > 0)
    hipLaunchKernelGGL(k_table_build, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, g,
                       reinterpret_cast<float4*>(voxel_pts), nullptr, reinterpret_cast<unsigned long long*>(status_dev),
                       1);
  O3DX_HIP(hipGetLastError());
  // occupancy not measured (-1): o3dx_estimate_normals_voxel skips its test
  const double gv[12] = {g.mnx + (double)g.kx0 * g.vs, g.mny, g.mnz, g.vs, (double)g.nx, (double)g.ny, (double)g.nz,
                         1.0, -1.0, (double)g.kx0, 0.0, (double)nvox};
  for (int k = 0; k < 12; ++k) geom_host[k] = gv[k];
  return 0;
}

int o3dx::voxel_down_sample_hooked(const float* xyz, int64_t n, const double* min_bound, const double* max_bound,
                             double voxel_size, int32_t* rep_idx, float* rep_xyz, int64_t* m_host, float* voxel_pts,
                             int64_t voxel_cells, double* geom, void* ws, size_t ws_bytes, void* stream,
                             VoxelHook hook, void* ctx, ZeroSpan extra_zero) {
  if (extra_zero.bytes && min_bound && max_bound)  // no bounds pass to clear it on the way
    O3DX_HIP(hipMemsetAsync(extra_zero.p, 0, extra_zero.bytes, as_stream(stream)));
  return voxel_impl(xyz, n, min_bound, max_bound, voxel_size, rep_idx, rep_xyz, m_host, nullptr, nullptr, voxel_pts,
                    voxel_cells, geom, ws, ws_bytes, stream, nullptr, hook, ctx, extra_zero);
}
