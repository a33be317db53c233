// grid.hip — spatial grid build, estimate_normals, batched kNN search.
//
// estimate_normals replaces o3d PointCloud.estimate_normals(param,
// fast_normal_computation=True) (reference open3dpypro/PointCloud.py:68-73,
// processors.py:243-249 CPUNormals, :267-303 TorchNormals' role).
// Per point: neighbour set (grid.hpp), Open3D's raw-moment float64 covariance
// (ComputeCovariance), FastEigen3x3 smallest eigenvector — both in float64,
// restated from Open3D geometry/EstimateNormals.cpp, utility/Eigen.cpp.
#include <type_traits>
#include <utility>

#include "grid.hpp"

namespace o3dx {

// ------------------------------------------------------------------ build
__global__ void __launch_bounds__(kBlock) k_grid_count(const float* __restrict__ xyz, int64_t n, GridView g,
                                                       int32_t* __restrict__ count, int32_t* __restrict__ cell,
                                                       int32_t* __restrict__ rank) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    int cx, cy, cz;
    grid_cell(g, x, y, z, cx, cy, cz);
    const int c = cell_index(g, cx, cy, cz);
    cell[i] = c;
    rank[i] = atomicAdd(&count[c], 1);
  }
}

__global__ void __launch_bounds__(kBlock) k_count_nonzero(const int32_t* __restrict__ count, int64_t nc,
                                                          unsigned long long* __restrict__ out) {
  int64_t local = 0;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x)
    local += count[c] != 0;
  __shared__ int64_t sh[kBlock / 64];
  local = wave_sum(local);
  if (lane_id() == 0) sh[threadIdx.x >> 6] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += sh[w];
    if (t) atomicAdd(out, (unsigned long long)t);
  }
}

__global__ void __launch_bounds__(kBlock) k_grid_scatter(const float* __restrict__ xyz, int64_t n,
                                                         const int32_t* __restrict__ cell,
                                                         const int32_t* __restrict__ rank,
                                                         const int32_t* __restrict__ start, float4* __restrict__ pts,
                                                         const float* __restrict__ extra_src,
                                                         float4* __restrict__ extra,
                                                         const int32_t* __restrict__ ids) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t pos = (int64_t)start[cell[i]] + rank[i];
    pts[pos] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], __int_as_float(ids ? ids[i] : (int)i));
    if (extra) extra[pos] = make_float4(extra_src[3 * i], extra_src[3 * i + 1], extra_src[3 * i + 2], 0.f);
  }
}

// Deterministic in-cell order (ascending original index; atomic ranks are
// not): every point counts the points of its cell with a smaller index and
// moves there — thread per point, O(cell size) reads each, all L2-local.
// Cells above kRankCell points are left to k_grid_big_cells (a workgroup per
// such cell, listed on the device by their first point): the cell's indices
// are staged in LDS tiles and each thread ranks its points against them, so a
// cell of c points costs c^2 / 1024 LDS reads per thread instead of a serial
// c^2 insertion sort (the round-2 cliff: 54 ms for a dense planted plane).
constexpr int kRankCell = 256;
constexpr int kBigTile = 8192;   // indices per LDS tile (32 KB)
constexpr int kBigBlock = 1024;

__global__ void __launch_bounds__(kBlock) k_grid_rank_fix(const float4* __restrict__ tmp,
                                                          const float4* __restrict__ tmp_extra, int64_t n,
                                                          const int32_t* __restrict__ cell,
                                                          const int32_t* __restrict__ start, float4* __restrict__ pts,
                                                          float4* __restrict__ extra, int32_t* __restrict__ big,
                                                          int32_t* __restrict__ nbig) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = tmp[p];
    const int i = __float_as_int(v.w);
    const int c = cell[i];
    const int s0 = start[c], s1 = start[c + 1];
    if (s1 - s0 > kRankCell) {  // the cell's workgroup places it
      if (p == s0) big[atomicAdd(nbig, 1)] = c;
      continue;
    }
    int r = 0;
    for (int q = s0; q < s1; ++q) r += __float_as_int(tmp[q].w) < i ? 1 : 0;
    const int dst = s0 + r;
    pts[dst] = v;
    if (extra) extra[dst] = tmp_extra[p];
  }
}

__global__ void __launch_bounds__(kBigBlock) k_grid_big_cells(const float4* __restrict__ tmp,
                                                              const float4* __restrict__ tmp_extra,
                                                              const int32_t* __restrict__ start,
                                                              const int32_t* __restrict__ big,
                                                              const int32_t* __restrict__ nbig,
                                                              float4* __restrict__ pts, float4* __restrict__ extra) {
  __shared__ int32_t ids[kBigTile];
  const int nb = *nbig;
  for (int b = blockIdx.x; b < nb; b += gridDim.x) {
    const int c = big[b];
    const int s0 = start[c], s1 = start[c + 1];
    const int m = s1 - s0;
    constexpr int kPer = 8;  // points ranked per thread per round
    for (int base = 0; base < m; base += kBigBlock * kPer) {
      int key[kPer], r[kPer];
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int j = base + threadIdx.x + u * kBigBlock;
        key[u] = j < m ? __float_as_int(tmp[s0 + j].w) : INT_MAX;
        r[u] = 0;
      }
      for (int t0 = 0; t0 < m; t0 += kBigTile) {
        const int tn = min(kBigTile, m - t0);
        __syncthreads();
        for (int j = threadIdx.x; j < tn; j += kBigBlock) ids[j] = __float_as_int(tmp[s0 + t0 + j].w);
        __syncthreads();
        for (int j = 0; j < tn; ++j) {
          const int id = ids[j];  // broadcast read
#pragma unroll
          for (int u = 0; u < kPer; ++u) r[u] += id < key[u] ? 1 : 0;
        }
      }
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int j = base + threadIdx.x + u * kBigBlock;
        if (j < m) {
          pts[s0 + r[u]] = tmp[s0 + j];
          if (extra) extra[s0 + r[u]] = tmp_extra[s0 + j];
        }
      }
    }
    __syncthreads();
  }
}

// Radix path of grid_build (large cell arrays: a surface cloud's fine grid
// holds up to cap_mult x n cells, 240 MB at C5, and the counting sort's
// returning atomics into it are random read-modify-writes of HBM lines):
// the cell keys are sorted with their point indices by a stable radix sort
// (in-cell order = ascending index, as the ordered counting path gives), the
// cell counts come from the runs of equal keys, and one gather writes the
// sorted points.  No atomics on the cell array.
__global__ void __launch_bounds__(kBlock) k_grid_keys(const float* __restrict__ xyz, int64_t n, GridView g,
                                                      uint32_t* __restrict__ key, int32_t* __restrict__ val) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int cx, cy, cz;
    grid_cell(g, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], cx, cy, cz);
    key[i] = (uint32_t)cell_index(g, cx, cy, cz);
    val[i] = (int32_t)i;
  }
}

__global__ void __launch_bounds__(kBlock) k_run_flags(const uint32_t* __restrict__ skey, int64_t n,
                                                      uint8_t* __restrict__ flags) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
    flags[p] = (p == 0 || skey[p] != skey[p - 1]) ? 1 : 0;
}

// runs[j] = the first sorted position of the j-th distinct key (nr of them)
__global__ void __launch_bounds__(kBlock) k_run_counts(const uint32_t* __restrict__ skey, const int32_t* __restrict__ runs,
                                                       const int64_t* __restrict__ nr, int64_t n,
                                                       int32_t* __restrict__ count) {
  const int64_t m = *nr;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = runs[j], b = j + 1 < m ? (int64_t)runs[j + 1] : n;
    count[skey[a]] = (int32_t)(b - a);
  }
}

// The dense start table straight from the runs (no per-cell count array and
// no scan over the cells): start[c] = the sorted position of the first run
// whose key is >= c (n past the last run), for every cell c in [0, nc].  Two
// passes: k_run_chunks (a thread per run) keys the runs (rkey[j]) and marks,
// for each chunk of kStartChunk cells, the first run at or after the chunk's
// first cell (cf[chunk]); k_start_fill (a block per chunk) stages the chunk's
// runs in LDS and writes its cells' starts, 16 consecutive cells per thread.
// Traffic: the runs once, the table once (written) — against a memset, a
// scattered count write and three passes of the scan over the cells before.
constexpr int kStartPer = 16;
constexpr int kStartChunk = kBlock * kStartPer;  // 4096 cells
__global__ void __launch_bounds__(kBlock) k_run_chunks(const uint32_t* __restrict__ skey, const int32_t* __restrict__ runs,
                                                       const int64_t* __restrict__ nr, int64_t nchunks,
                                                       uint32_t* __restrict__ rkey, int32_t* __restrict__ cf) {
  const int64_t m = *nr;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = skey[runs[j]];
    rkey[j] = k;
    // chunks c with key[j - 1] < c * kStartChunk <= key[j] start at run j
    const int64_t c0 = j == 0 ? 0 : (int64_t)(skey[runs[j - 1]] / kStartChunk) + 1;
    const int64_t c1 = k / kStartChunk;
    for (int64_t c = c0; c <= c1; ++c) cf[c] = (int32_t)j;
    if (j == m - 1)  // the chunks after the last run's: every cell there starts at n
      for (int64_t c = c1 + 1; c <= nchunks; ++c) cf[c] = (int32_t)m;
  }
}

__global__ void __launch_bounds__(kBlock) k_start_fill(const uint32_t* __restrict__ rkey,
                                                       const int32_t* __restrict__ runs,
                                                       const int64_t* __restrict__ nr, const int32_t* __restrict__ cf,
                                                       int64_t nc, int64_t n, int32_t* __restrict__ start) {
  __shared__ uint32_t key[kStartChunk];
  __shared__ int32_t pos[kStartChunk + 1];
  const int64_t m = *nr;
  const int64_t base = (int64_t)blockIdx.x * kStartChunk;
  const int j0 = cf[blockIdx.x], j1 = cf[blockIdx.x + 1];
  const int cnt = j1 - j0;  // runs keyed inside this chunk (<= kStartChunk: distinct keys)
  for (int t = threadIdx.x; t < cnt; t += kBlock) {
    key[t] = rkey[j0 + t];
    pos[t] = runs[j0 + t];
  }
  if (threadIdx.x == 0) pos[cnt] = j1 < m ? runs[j1] : (int32_t)n;
  __syncthreads();
  const int64_t c0 = base + (int64_t)threadIdx.x * kStartPer;
  if (c0 > nc) return;
  // first staged run with key >= c0, then forward over the thread's cells
  int lo = 0, hi = cnt;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)key[mid] < c0) lo = mid + 1;
    else hi = mid;
  }
  int32_t v[kStartPer];
#pragma unroll
  for (int i = 0; i < kStartPer; ++i) {
    while (lo < cnt && (int64_t)key[lo] < c0 + i) ++lo;
    v[i] = pos[lo];
  }
  if (c0 + kStartPer <= nc + 1) {
    int4* o = reinterpret_cast<int4*>(start + c0);  // c0 is a multiple of 16: 64-B aligned
#pragma unroll
    for (int i = 0; i < kStartPer / 4; ++i) o[i] = make_int4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
  } else {
#pragma unroll
    for (int i = 0; i < kStartPer; ++i)
      if (c0 + i <= nc) start[c0 + i] = v[i];
  }
}

__global__ void __launch_bounds__(kBlock) k_grid_gather(const float* __restrict__ xyz, int64_t n,
                                                        const int32_t* __restrict__ sval, float4* __restrict__ pts,
                                                        const float* __restrict__ extra_src, float4* __restrict__ extra,
                                                        const int32_t* __restrict__ ids) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = sval[p];
    pts[p] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], __int_as_float(ids ? ids[i] : (int)i));
    if (extra) extra[p] = make_float4(extra_src[3 * i], extra_src[3 * i + 1], extra_src[3 * i + 2], 0.f);
  }
}

// the surface test of a large cloud on every `stride`-th point: no returning
// atomics, no per-point writes (a surface puts hundreds of points in each
// coarse cell, and the full count's returning atomics queue on those cells)
__global__ void __launch_bounds__(kBlock) k_grid_count_sample(const float* __restrict__ xyz, int64_t n, GridView g,
                                                              int stride, int32_t* __restrict__ count) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t * stride < n; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t * stride;
    int cx, cy, cz;
    grid_cell(g, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], cx, cy, cz);
    atomicAdd(&count[cell_index(g, cx, cy, cz)], 1);
  }
}
constexpr int kSampleStride = 8;

// from this many cells (and points) the fine pass takes the radix path
constexpr int64_t kRadixMinCells = (int64_t)1 << 24;
constexpr int64_t kRadixMinPoints = (int64_t)1 << 20;

// cell-index capacity: cap_mult cells per point (the dense start table costs
// 8 B per cell: count + start)
static int64_t cap_cells(int64_t n, int cap_mult) { return std::max<int64_t>((int64_t)cap_mult * n, 4096); }

struct GridLayout {
  size_t pts, extra, tmp, tmp_extra, count, start, cell, rank, scan, aabb, mm, scratch, total;
};

static GridLayout grid_layout(int64_t n, int cap_mult) {
  n = std::max<int64_t>(n, 1);
  GridLayout L;
  size_t o = 0;
  auto put = [&](size_t bytes) {
    size_t at = o;
    o += Arena::align(bytes + 1);
    return at;
  };
  int64_t cc = cap_cells(n, cap_mult);
  L.pts = put(n * sizeof(float4));
  L.extra = put(n * sizeof(float4));
  L.tmp = put(n * sizeof(float4));
  L.tmp_extra = put(n * sizeof(float4));
  L.count = put((cc + 1) * sizeof(int32_t));
  L.start = put((cc + 1) * sizeof(int32_t));
  L.cell = put(n * sizeof(int32_t));
  L.rank = put(n * sizeof(int32_t));
  L.scan = put(scan_workspace_ints(cc + 1) * sizeof(int32_t));
  L.aabb = put(aabb_ws_bytes(n));
  L.mm = put(8 * sizeof(double));
  L.scratch = put(8 * sizeof(int64_t));
  L.total = o;
  return L;
}

size_t grid_ws_bytes(int64_t n, int cap_mult) { return grid_layout(n, cap_mult).total; }

// Test / profiling hooks.  They are thread-local: a hook set on one host
// thread affects only the launches that thread makes, so the library stays
// re-entrant across threads; unset they cost a null test.
// Debug-only search statistics (o3dx_search_stats): the one place the library
// allocates device memory, and only after o3dx_set_search_stats(1).
static thread_local unsigned long long* g_stats = nullptr;
static thread_local bool g_stats_on = false;
unsigned long long* search_stats_ptr() { return g_stats_on ? g_stats : nullptr; }

// Test hook (o3dx_set_debug_neighbors): caller-owned (rows, k) buffer.
static thread_local int32_t* g_dbg_nbr = nullptr;
static thread_local int64_t g_dbg_rows = 0;
static thread_local int g_dbg_k = 0;
static int32_t* debug_nbr(int kneed, int64_t rows) {
  return (g_dbg_nbr && kneed == g_dbg_k && rows <= g_dbg_rows) ? g_dbg_nbr : nullptr;
}


static void dims_for(const double mn[3], const double mx[3], double h, int64_t d[3]) {
  for (int a = 0; a < 3; ++a) d[a] = (int64_t)std::floor(std::max(0.0, mx[a] - mn[a]) / h) + 1;
}

// size of the cell index space for dims d
static int64_t cell_space(const int64_t d[3], bool blocked) {
  if (!blocked) return d[0] * d[1] * d[2];
  return ((d[0] + 7) / 8) * ((d[1] + 7) / 8) * ((d[2] + 7) / 8) * 512;
}

int grid_build(const float* xyz, int64_t n, double target_occ, double min_h, void* ws, size_t ws_bytes,
               hipStream_t s, GridBuild* out, float4* extra_sorted, const float* extra_src, bool blocked,
               int cap_mult, bool ordered, const int32_t* ids, double max_h) {
  if (ids) ordered = false;  // the in-cell ranking reads the cell of point w
  GridLayout L = grid_layout(n, cap_mult);
  if (ws_bytes < L.total) return fail(O3DX_ENOMEM, "grid workspace too small (need %zu)", L.total);
  char* w = (char*)ws;
  GridBuild& G = *out;
  G.pts = (float4*)(w + L.pts);
  G.start = (int32_t*)(w + L.start);
  G.count = (int32_t*)(w + L.count);
  G.cell = (int32_t*)(w + L.cell);
  G.rank = (int32_t*)(w + L.rank);
  G.scan_tmp = (int32_t*)(w + L.scan);
  G.aabb_ws = w + L.aabb;
  G.mm = (double*)(w + L.mm);
  G.scratch = (int64_t*)(w + L.scratch);
  G.cap_cells = cap_cells(std::max<int64_t>(n, 1), cap_mult);
  if (!extra_sorted && extra_src) extra_sorted = (float4*)(w + L.extra);
  G.extra = extra_sorted;

  double mm[6];
  O3DX_TRY(aabb_device(xyz, n, G.mm, G.aabb_ws, s));
  O3DX_TRY(read_back(mm, G.mm, 6 * sizeof(double), s));
  std::memcpy(G.mm_host, mm, sizeof(mm));
  const double mn[3] = {mm[0], mm[1], mm[2]}, mx[3] = {mm[3], mm[4], mm[5]};
  double ext[3], maxabs = 0, maxext = 0;
  for (int a = 0; a < 3; ++a) {
    ext[a] = std::max(0.0, mx[a] - mn[a]);
    maxabs = std::max(maxabs, std::max(std::fabs(mn[a]), std::fabs(mx[a])));
    maxext = std::max(maxext, ext[a]);
  }
  // cell size from the density over the "thick" dimensions of the box
  const double nn = (double)std::max<int64_t>(n, 1);
  double h = maxext > 0 ? maxext : 1.0;
  for (int it = 0; it < 4 && maxext > 0; ++it) {
    double vol = 1.0;
    int d = 0;
    for (int a = 0; a < 3; ++a)
      if (ext[a] > h * 0.5) {
        vol *= ext[a];
        ++d;
      }
    if (d == 0) break;
    double hn = std::pow(vol * target_occ / nn, 1.0 / d);
    if (std::fabs(hn - h) <= 1e-9 * h) break;
    h = hn;
  }
  if (min_h > 0) h = std::max(h, min_h);
  if (max_h > 0) h = std::min(h, max_h);
  if (!(h > 0) || !std::isfinite(h)) h = 1.0;
  auto fit_cap = [&](double hh) {
    int64_t d[3];
    for (int guard = 0; guard < 64; ++guard) {
      dims_for(mn, mx, hh, d);
      double cells = (double)cell_space(d, blocked);
      if (cells <= (double)G.cap_cells) break;
      hh *= std::cbrt(cells / (double)G.cap_cells) * 1.01;
    }
    return hh;
  };
  h = fit_cap(h);

  for (int pass = 0; pass < 2; ++pass) {
    int64_t d[3];
    dims_for(mn, mx, h, d);
    GridView& g = G.view;
    g.pts = G.pts;
    g.start = G.start;
    g.ox = (float)mn[0];
    g.oy = (float)mn[1];
    g.oz = (float)mn[2];
    g.h = (float)h;
    g.inv_h = (float)(1.0 / h);
    g.nx = (int)d[0];
    g.ny = (int)d[1];
    g.nz = (int)d[2];
    g.n = n;
    g.stats = search_stats_ptr();
    // assignment error of a float32 cell computation, both sides of a face
    g.slack = (float)(32.0 * std::ldexp(1.0, -24) * (maxabs + maxext) + 1e-6 * h);
    g.blocked = blocked ? 1 : 0;
    g.bnx = (int)((d[0] + 7) / 8);
    g.bny = (int)((d[1] + 7) / 8);
    const int64_t nc = cell_space(d, blocked);
    // the fine pass of a surface cloud (pass 1) over a large cell array: the
    // radix path (O3DX_GRID_ATOMIC: tests, the counting path instead)
    if (pass == 1 && nc >= kRadixMinCells && n >= kRadixMinPoints && n < INT32_MAX && !getenv("O3DX_GRID_ATOMIC")) {
      int bits = 1;
      while (bits < 32 && ((int64_t)1 << bits) < nc) ++bits;
      const size_t need = cell_sort_temp_bytes(n, bits);
      const size_t avail = L.count - L.tmp_extra;  // tmp_extra: unused on this path
      if (need <= avail) {
        KTimer kt_sort("grid_sort", s);
        uint32_t* key = reinterpret_cast<uint32_t*>(G.cell);
        int32_t* val = G.rank;
        uint32_t* skey = reinterpret_cast<uint32_t*>(w + L.tmp);
        int32_t* sval = reinterpret_cast<int32_t*>(skey + n);
        const unsigned gn = grid_for(n, kBlock, 8192);
        hipLaunchKernelGGL(k_grid_keys, dim3(gn), dim3(kBlock), 0, s, xyz, n, g, key, val);
        O3DX_TRY(cell_sort(key, skey, val, sval, n, bits, w + L.tmp_extra, avail, s));
        // the runs of equal keys -> cell counts -> starts
        uint8_t* flags = reinterpret_cast<uint8_t*>(G.rank);  // val is dead after the sort
        int32_t* runs = G.cell;                                // so is key
        int64_t* nr = G.scratch + 2;
        hipLaunchKernelGGL(k_run_flags, dim3(gn), dim3(kBlock), 0, s, skey, n, flags);
        O3DX_TRY(compact_flags(flags, n, runs, nullptr, nr, G.scan_tmp, s));
        if (getenv("O3DX_GRID_SCAN_STARTS")) {  // the count + scan form (A/B, tests)
          O3DX_HIP(hipMemsetAsync(G.count, 0, (nc + 1) * sizeof(int32_t), s));
          hipLaunchKernelGGL(k_run_counts, dim3(gn), dim3(kBlock), 0, s, skey, runs, nr, n, G.count);
          O3DX_TRY(exclusive_scan_i32(G.count, G.start, nc, G.scan_tmp, s));
        } else {
          // run keys in the count array (m <= n <= its cells), chunk heads in
          // the scan scratch (>= one int per 4096 cells + 64)
          const int64_t nchunks = (nc + 1 + kStartChunk - 1) / kStartChunk;
          uint32_t* rkey = reinterpret_cast<uint32_t*>(G.count);
          int32_t* cf = G.scan_tmp;
          hipLaunchKernelGGL(k_run_chunks, dim3(gn), dim3(kBlock), 0, s, skey, runs, nr, nchunks, rkey, cf);
          hipLaunchKernelGGL(k_start_fill, dim3((unsigned)nchunks), dim3(kBlock), 0, s, rkey, runs, nr, cf, nc, n,
                             G.start);
        }
        hipLaunchKernelGGL(k_grid_gather, dim3(gn), dim3(kBlock), 0, s, xyz, n, sval, G.pts, extra_src, extra_sorted,
                           ids);
        O3DX_HIP(hipGetLastError());
        break;
      }
    }
    KTimer kt_count("grid_count", s);
    bool sampled = false;
    if (pass == 0 && n >= kRadixMinPoints && !getenv("O3DX_GRID_ATOMIC")) {
      // large clouds: the surface test on a 1/8 sample (the occupied cells it
      // sees are a lower bound, so its mean occupancy an upper bound of the
      // cloud's); a surface goes straight to its fine pass, a volume to the
      // full count at this h below
      unsigned long long occ = 0;
      O3DX_HIP(hipMemsetAsync(G.count, 0, (nc + 1) * sizeof(int32_t), s));
      O3DX_HIP(hipMemsetAsync(G.scratch, 0, sizeof(int64_t), s));
      hipLaunchKernelGGL(k_grid_count_sample, dim3(grid_for((n + kSampleStride - 1) / kSampleStride, kBlock, 8192)),
                         dim3(kBlock), 0, s, xyz, n, g, kSampleStride, G.count);
      hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(nc, kBlock, 1024)), dim3(kBlock), 0, s, G.count, nc,
                         (unsigned long long*)G.scratch);
      O3DX_TRY(read_back(&occ, G.scratch, sizeof(occ), s));
      const double mean_occ = occ ? nn / (double)occ : nn;
      if (mean_occ > 2.5 * target_occ) {
        double hn = h * std::sqrt(target_occ / mean_occ);
        if (min_h > 0) hn = std::max(hn, min_h);
        hn = fit_cap(hn);
        if (hn < h * 0.9) {
          h = hn;
          continue;
        }
      }
      sampled = true;
    }
    O3DX_HIP(hipMemsetAsync(G.count, 0, (nc + 1) * sizeof(int32_t), s));
    if (n > 0)
      hipLaunchKernelGGL(k_grid_count, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, g, G.count,
                         G.cell, G.rank);
    if (pass == 0 && n > 64 && !sampled) {
      // surface-like clouds: occupied cells are far denser than the box average
      unsigned long long occ = 0;
      O3DX_HIP(hipMemsetAsync(G.scratch, 0, sizeof(int64_t), s));
      hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(nc, kBlock, 1024)), dim3(kBlock), 0, s, G.count, nc,
                         (unsigned long long*)G.scratch);
      O3DX_TRY(read_back(&occ, G.scratch, sizeof(occ), s));
      double mean_occ = occ ? nn / (double)occ : nn;
      if (mean_occ > 2.5 * target_occ) {
        double hn = h * std::sqrt(target_occ / mean_occ);
        if (min_h > 0) hn = std::max(hn, min_h);
        hn = fit_cap(hn);
        if (hn < h * 0.9) {
          h = hn;
          continue;
        }
      }
    }
    kt_count.stop();
    KTimer kt_sort("grid_sort", s);
    O3DX_TRY(exclusive_scan_i32(G.count, G.start, nc, G.scan_tmp, s));
    if (n > 0 && !ordered) {  // cell order only (the in-cell order is the atomic ranks')
      hipLaunchKernelGGL(k_grid_scatter, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, G.cell, G.rank,
                         G.start, G.pts, extra_src, extra_sorted, ids);
    } else if (n > 0) {
      float4* tmp = (float4*)(w + L.tmp);
      float4* tmp_extra = extra_sorted ? (float4*)(w + L.tmp_extra) : nullptr;
      hipLaunchKernelGGL(k_grid_scatter, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, G.cell, G.rank,
                         G.start, tmp, extra_src, tmp_extra, (const int32_t*)nullptr);
      // the big-cell list reuses the per-point rank array (free after the scatter)
      int32_t* nbig = reinterpret_cast<int32_t*>(G.scratch + 1);
      O3DX_HIP(hipMemsetAsync(nbig, 0, sizeof(int32_t), s));
      hipLaunchKernelGGL(k_grid_rank_fix, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, tmp, tmp_extra, n,
                         G.cell, G.start, G.pts, extra_sorted, G.rank, nbig);
      hipLaunchKernelGGL(k_grid_big_cells, dim3(512), dim3(kBigBlock), 0, s, tmp, tmp_extra, G.start, G.rank, nbig,
                         G.pts, extra_sorted);
    }
    O3DX_HIP(hipGetLastError());
    break;
  }
  return 0;
}


// ------------------------------------------------------------- chunk plan
// Queries = the grid's own (cell-sorted) points, so the queries of grid row
// k = (y, z) are the contiguous range [start[k nx], start[(k+1) nx]).  Rows
// of >= qcap queries are cut into chunks of qcap; within a group of
// kChunkRows consecutive rows of one z slab, shorter rows are merged with
// their successors (contiguous in memory) while the chunk stays <= qcap
// queries — on a surface seen edge-on every row holds only a few points.
// One thread per group; no host synchronisation: the caller launches `upper`
// blocks, the slots past the real chunk count hold n (empty chunks) and slot
// upper+1 holds the count.
constexpr int kChunkRows = 10;  // box rows (kChunkRows + 2) x 3 <= kMaxTileRows

template <bool EMIT>
__global__ void k_group_chunks(const int32_t* __restrict__ start, int nx, int ny, int nz, int qcap,
                               int32_t* __restrict__ cnt_or_off, int32_t* __restrict__ chunk_starts) {
  const int gy = (ny + kChunkRows - 1) / kChunkRows;
  const int64_t grp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (grp >= (int64_t)gy * nz) return;
  const int z = (int)(grp / gy), y0 = (int)(grp % gy) * kChunkRows, y1 = min(y0 + kChunkRows, ny);
  int32_t bnd[kChunkRows + 1];
#pragma unroll
  for (int j = 0; j <= kChunkRows; ++j)
    bnd[j] = start[(int64_t)min(y0 + j, y1) * nx + (int64_t)ny * nx * z];
  int cnt = 0, o = EMIT ? cnt_or_off[grp] : 0;
  int open_start = -1, open_len = 0;
#pragma unroll
  for (int j = 0; j < kChunkRows; ++j) {
    const int32_t a = bnd[j], len = bnd[j + 1] - a;
    if (len == 0) continue;
    if (open_start >= 0 && (len >= qcap || open_len + len > qcap)) {
      if (EMIT) chunk_starts[o++] = open_start;
      ++cnt;
      open_start = -1;
      open_len = 0;
    }
    if (len >= qcap) {
      for (int32_t p = a; p < a + len; p += qcap) {
        if (EMIT) chunk_starts[o++] = p;
        ++cnt;
      }
      continue;
    }
    if (open_start < 0) open_start = a;
    open_len += len;
  }
  if (open_start >= 0) {
    if (EMIT) chunk_starts[o] = open_start;
    ++cnt;
  }
  if (!EMIT) cnt_or_off[grp] = cnt;
}

__global__ void k_chunk_tail(const int32_t* __restrict__ offs, int64_t ngroups, int64_t n, int64_t upper,
                             int32_t* __restrict__ chunk_starts) {
  const int64_t total = offs[ngroups];
  for (int64_t c = total + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c <= upper;
       c += (int64_t)gridDim.x * blockDim.x)
    chunk_starts[c] = (int32_t)n;
  if (blockIdx.x == 0 && threadIdx.x == 0) chunk_starts[upper + 1] = (int32_t)total;
}

int64_t chunk_plan_upper(int64_t n, const GridView& g, int qcap) {
  return (n + qcap - 1) / qcap + (int64_t)g.ny * g.nz;
}

size_t chunk_plan_ws_bytes(int64_t n, int64_t rows) {
  rows = std::max<int64_t>(rows, 1);  // bounds the number of row groups too
  (void)n;
  return 2 * Arena::align((rows + 2) * 4) + Arena::align(scan_workspace_ints(rows + 1) * 4 + 1) + 1024;
}

int chunk_plan(int64_t n, const GridView& g, int qcap, int32_t* chunk_starts, void* ws, size_t ws_bytes,
               hipStream_t s) {
  const int64_t rows = (int64_t)g.ny * g.nz;
  if (ws_bytes < chunk_plan_ws_bytes(n, rows)) return fail(O3DX_ENOMEM, "chunk plan workspace too small");
  Arena ar(ws, ws_bytes);
  const int64_t ngroups = (int64_t)((g.ny + kChunkRows - 1) / kChunkRows) * g.nz;
  int32_t* cnt = ar.take<int32_t>(ngroups + 1);
  int32_t* offs = ar.take<int32_t>(ngroups + 1);
  int32_t* tmp = ar.take<int32_t>(scan_workspace_ints(ngroups + 1));
  const int64_t upper = chunk_plan_upper(n, g, qcap);
  const unsigned gg = (unsigned)((ngroups + 255) / 256);
  hipLaunchKernelGGL(k_group_chunks<false>, dim3(gg), dim3(256), 0, s, g.start, g.nx, g.ny, g.nz, qcap, cnt,
                     (int32_t*)nullptr);
  O3DX_TRY(exclusive_scan_i32(cnt, offs, ngroups, tmp, s));
  hipLaunchKernelGGL(k_group_chunks<true>, dim3(gg), dim3(256), 0, s, g.start, g.nx, g.ny, g.nz, qcap, offs,
                     chunk_starts);
  hipLaunchKernelGGL(k_chunk_tail, dim3(256), dim3(256), 0, s, offs, ngroups, n, upper, chunk_starts);
  O3DX_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------- FastEigen3x3 (f64)
__device__ __forceinline__ void dcross(const double u[3], const double v[3], double o[3]) {
  o[0] = u[1] * v[2] - u[2] * v[1];
  o[1] = u[2] * v[0] - u[0] * v[2];
  o[2] = u[0] * v[1] - u[1] * v[0];
}
__device__ __forceinline__ double ddot(const double u[3], const double v[3]) {
  return (u[0] * v[0] + u[1] * v[1]) + u[2] * v[2];
}

// Open3D ComputeEigenvector0
__device__ void eigvec0(const double A[3][3], double e, double out[3]) {
  double r0[3] = {A[0][0] - e, A[0][1], A[0][2]};
  double r1[3] = {A[0][1], A[1][1] - e, A[1][2]};
  double r2[3] = {A[0][2], A[1][2], A[2][2] - e};
  double a[3], b[3], c[3];
  dcross(r0, r1, a);
  dcross(r0, r2, b);
  dcross(r1, r2, c);
  double d0 = ddot(a, a), d1 = ddot(b, b), d2 = ddot(c, c);
  double dmax = d0;
  int imax = 0;
  if (d1 > dmax) {
    dmax = d1;
    imax = 1;
  }
  if (d2 > dmax) imax = 2;
  if (imax == 0) {
    double s = sqrt(d0);
    out[0] = a[0] / s; out[1] = a[1] / s; out[2] = a[2] / s;
  } else if (imax == 1) {
    double s = sqrt(d1);
    out[0] = b[0] / s; out[1] = b[1] / s; out[2] = b[2] / s;
  } else {
    double s = sqrt(d2);
    out[0] = c[0] / s; out[1] = c[1] / s; out[2] = c[2] / s;
  }
}

// Open3D ComputeEigenvector1
__device__ void eigvec1(const double A[3][3], const double e0[3], double e1v, double out[3]) {
  double U[3], V[3];
  if (fabs(e0[0]) > fabs(e0[1])) {
    double inv = 1.0 / sqrt(e0[0] * e0[0] + e0[2] * e0[2]);
    U[0] = -e0[2] * inv; U[1] = 0; U[2] = e0[0] * inv;
  } else {
    double inv = 1.0 / sqrt(e0[1] * e0[1] + e0[2] * e0[2]);
    U[0] = 0; U[1] = e0[2] * inv; U[2] = -e0[1] * inv;
  }
  dcross(e0, U, V);
  double AU[3] = {A[0][0] * U[0] + A[0][1] * U[1] + A[0][2] * U[2], A[0][1] * U[0] + A[1][1] * U[1] + A[1][2] * U[2],
                  A[0][2] * U[0] + A[1][2] * U[1] + A[2][2] * U[2]};
  double AV[3] = {A[0][0] * V[0] + A[0][1] * V[1] + A[0][2] * V[2], A[0][1] * V[0] + A[1][1] * V[1] + A[1][2] * V[2],
                  A[0][2] * V[0] + A[1][2] * V[1] + A[2][2] * V[2]};
  double m00 = U[0] * AU[0] + U[1] * AU[1] + U[2] * AU[2] - e1v;
  double m01 = U[0] * AV[0] + U[1] * AV[1] + U[2] * AV[2];
  double m11 = V[0] * AV[0] + V[1] * AV[1] + V[2] * AV[2] - e1v;
  double a00 = fabs(m00), a01 = fabs(m01), a11 = fabs(m11);
  if (a00 >= a11) {
    if (fmax(a00, a01) > 0) {
      if (a00 >= a01) {
        m01 /= m00; m00 = 1 / sqrt(1 + m01 * m01); m01 *= m00;
      } else {
        m00 /= m01; m01 = 1 / sqrt(1 + m00 * m00); m00 *= m01;
      }
      for (int i = 0; i < 3; ++i) out[i] = m01 * U[i] - m00 * V[i];
    } else {
      for (int i = 0; i < 3; ++i) out[i] = U[i];
    }
  } else {
    if (fmax(a11, a01) > 0) {
      if (a11 >= a01) {
        m01 /= m11; m11 = 1 / sqrt(1 + m01 * m01); m01 *= m11;
      } else {
        m11 /= m01; m01 = 1 / sqrt(1 + m11 * m11); m11 *= m01;
      }
      for (int i = 0; i < 3; ++i) out[i] = m11 * U[i] - m01 * V[i];
    } else {
      for (int i = 0; i < 3; ++i) out[i] = U[i];
    }
  }
}

// Open3D FastEigen3x3 (Eberly's robust symmetric 3x3 solver): smallest eigenvector.
// c = {xx, xy, xz, yy, yz, zz}
__device__ void fast_eigen3x3(const double c[6], double out[3]) {
  double A[3][3] = {{c[0], c[1], c[2]}, {c[1], c[3], c[4]}, {c[2], c[4], c[5]}};
  double max_coeff = A[0][0];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) max_coeff = fmax(max_coeff, A[i][j]);
  if (max_coeff == 0) {
    out[0] = out[1] = out[2] = 0;
    return;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[i][j] /= max_coeff;
  double norm = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
  if (norm > 0) {
    double q = (A[0][0] + A[1][1] + A[2][2]) / 3;
    double b00 = A[0][0] - q, b11 = A[1][1] - q, b22 = A[2][2] - q;
    double p = sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2) / 6);
    double c00 = b11 * b22 - A[1][2] * A[1][2];
    double c01 = A[0][1] * b22 - A[1][2] * A[0][2];
    double c02 = A[0][1] * A[1][2] - b11 * A[0][2];
    double det = (b00 * c00 - A[0][1] * c01 + A[0][2] * c02) / (p * p * p);
    double half_det = fmin(fmax(det * 0.5, -1.0), 1.0);
    double angle = acos(half_det) / (double)3;
    const double two_thirds_pi = 2.09439510239319549;
    double beta2 = cos(angle) * 2;
    double beta0 = cos(angle + two_thirds_pi) * 2;
    double beta1 = -(beta0 + beta2);
    double ev0 = q + p * beta0, ev1 = q + p * beta1, ev2 = q + p * beta2;
    double ea[3], eb[3];
    if (half_det >= 0) {
      eigvec0(A, ev2, ea);
      if (ev2 < ev0 && ev2 < ev1) {
        out[0] = ea[0]; out[1] = ea[1]; out[2] = ea[2];
        return;
      }
      eigvec1(A, ea, ev1, eb);
      if (ev1 < ev0 && ev1 < ev2) {
        out[0] = eb[0]; out[1] = eb[1]; out[2] = eb[2];
        return;
      }
      dcross(eb, ea, out);  // evec0 = evec1 x evec2
    } else {
      eigvec0(A, ev0, ea);
      if (ev0 < ev1 && ev0 < ev2) {
        out[0] = ea[0]; out[1] = ea[1]; out[2] = ea[2];
        return;
      }
      eigvec1(A, ea, ev1, eb);
      if (ev1 < ev0 && ev1 < ev2) {
        out[0] = eb[0]; out[1] = eb[1]; out[2] = eb[2];
        return;
      }
      dcross(ea, eb, out);  // evec2 = evec0 x evec1
    }
  } else {
    if (A[0][0] < A[1][1] && A[0][0] < A[2][2]) {
      out[0] = 1; out[1] = 0; out[2] = 0;
    } else if (A[1][1] < A[0][0] && A[1][1] < A[2][2]) {
      out[0] = 0; out[1] = 1; out[2] = 0;
    } else {
      out[0] = 0; out[1] = 0; out[2] = 1;
    }
  }
}

struct MomAcc {
  double m[9];
  __device__ void zero() {
#pragma unroll
    for (int j = 0; j < 9; ++j) m[j] = 0.0;
  }
  __device__ void init(const float4&, float, int) {}
  // Open3D ComputeCovariance cumulant order.  The coordinates are float32
  // values, so every product is exact in float64 and fma(x, y, m) rounds
  // exactly as m + x * y: one instruction instead of two (the build keeps
  // -ffp-contract=off).
  __device__ void add(double x, double y, double z) {
    m[0] += x;
    m[1] += y;
    m[2] += z;
    m[3] = fma(x, x, m[3]);
    m[4] = fma(x, y, m[4]);
    m[5] = fma(x, z, m[5]);
    m[6] = fma(y, y, m[6]);
    m[7] = fma(y, z, m[7]);
    m[8] = fma(z, z, m[8]);
  }
  __device__ void cov(int k, double c[6]) const {
    double u[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) u[j] = m[j] / (double)k;
    c[0] = u[3] - u[0] * u[0];
    c[3] = u[6] - u[1] * u[1];
    c[5] = u[8] - u[2] * u[2];
    c[1] = u[4] - u[0] * u[1];
    c[2] = u[5] - u[0] * u[2];
    c[4] = u[7] - u[1] * u[2];
  }
};

// Exact-sum form of MomAcc for the sorted-grid kernels: each moment is a
// double-double (h, l) grown by TwoSum.  The terms are exact (coordinates
// are float32 values, their pairwise products fit float64), and while a
// neighbourhood's non-zero coordinates lie within a factor 2^22 of each other
// every (h, l) stays the exact partial sum, so h + l rounded once is the
// correctly rounded exact sum: the same bits in ANY summation order.  The
// sorted grid's scan order depends on its cell geometry, which depends on the
// cloud given (a slab's own + halo points in the multi-GPU path, the whole
// cloud on one GPU); with exact sums the normals do not.  (The voxel-table
// kernels scan the global voxel grid in a fixed stencil order and keep the
// plain sums.)
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

struct MomAccDD {
  double m[9];  // h parts; cov() reads h + l
  double l[9];
  __device__ void zero() {
#pragma unroll
    for (int j = 0; j < 9; ++j) m[j] = l[j] = 0.0;
  }
  __device__ void init(const float4&, float, int) {}
  __device__ __forceinline__ void put(int j, double t) {
    double s, e;
    two_sum(m[j], t, s, e);
    m[j] = s;
    l[j] += e;
  }
  __device__ void add(double x, double y, double z) {
    put(0, x);
    put(1, y);
    put(2, z);
    put(3, x * x);
    put(4, x * y);
    put(5, x * z);
    put(6, y * y);
    put(7, y * z);
    put(8, z * z);
  }
  __device__ void cov(int k, double c[6]) const {
    MomAcc a;
#pragma unroll
    for (int j = 0; j < 9; ++j) a.m[j] = m[j] + l[j];
    a.cov(k, c);
  }
};

// The same correctly rounded exact sums as MomAccDD at half its cost, for a
// selection whose members all lie within sqrt(r2) of the query q: each moment
// starts at an anchor A (a power of two >= 4 x the bound on the sum of |terms|
// of up to kmax neighbours, from |q| + sqrt(r2) per axis), so every partial
// sum stays in [A/2, 2A) and is at least as large as any term — Fast2Sum (3
// flops) then gives each addition's exact error, where MomAccDD's TwoSum
// takes 6.  m - A is exact (Sterbenz); (m - A) + l, rounded once, is the
// correctly rounded exact sum under MomAccDD's condition (non-zero
// coordinates within a factor 2^22: the errors then fit l exactly), so the
// bits equal MomAccDD's and every other exact path's.
struct MomAccA {
  double m[9], l[9], a[9];
  __device__ void zero() {
#pragma unroll
    for (int j = 0; j < 9; ++j) m[j] = l[j] = a[j] = 0.0;
  }
  __device__ void init(const float4& q, float r2, int kmax) {
    const double r = sqrt((double)r2) * (1.0 + 1e-6) + 1e-30;
    const double X = fabs((double)q.x) + r, Y = fabs((double)q.y) + r, Z = fabs((double)q.z) + r;
    const double b[9] = {X, Y, Z, X * X, X * Y, X * Z, Y * Y, Y * Z, Z * Z};
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      a[j] = ldexp(1.0, ilogb((double)kmax * b[j]) + 3);  // >= 4 kmax b (ilogb floors)
      m[j] = a[j];
    }
  }
  __device__ __forceinline__ void put(int j, double t) {
    const double s = m[j] + t;
    l[j] += t - (s - m[j]);
    m[j] = s;
  }
  __device__ void add(double x, double y, double z) {
    put(0, x);
    put(1, y);
    put(2, z);
    put(3, x * x);
    put(4, x * y);
    put(5, x * z);
    put(6, y * y);
    put(7, y * z);
    put(8, z * z);
  }
  __device__ void cov(int k, double c[6]) const {
    MomAcc acc;
#pragma unroll
    for (int j = 0; j < 9; ++j) acc.m[j] = (m[j] - a[j]) + l[j];
    acc.cov(k, c);
  }
};

// Open3D ComputeCovariance on float64 storage: the nine cumulants summed in
// the neighbours' result order (nanoflann's: (d^2, index) ascending), each
// product rounded then added (the build's -ffp-contract=off) — the float64
// coordinates' products are not exact, so the order and the roundings are
// Open3D's own, for the same bits.
struct MomAccSeq {
  double m[9];
  __device__ void zero() {
#pragma unroll
    for (int j = 0; j < 9; ++j) m[j] = 0.0;
  }
  __device__ void add(double x, double y, double z) {
    m[0] += x;
    m[1] += y;
    m[2] += z;
    m[3] += x * x;
    m[4] += x * y;
    m[5] += x * z;
    m[6] += y * y;
    m[7] += y * z;
    m[8] += z * z;
  }
  __device__ void cov(int k, double c[6]) const {
    MomAcc a;
#pragma unroll
    for (int j = 0; j < 9; ++j) a.m[j] = m[j];
    a.cov(k, c);
  }
};

// wave-wide exact sum of exact terms (the same condition as MomAccDD): an
// xor tree of (h, l) pairs joined by TwoSum, h + l rounded once
__device__ __forceinline__ double wave_sum_exact(double t) {
  double h = t, l = 0.0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double h2 = __shfl_xor(h, o, 64), l2 = __shfl_xor(l, o, 64);
    double s, e;
    two_sum(h, h2, s, e);
    h = s;
    l = (l + l2) + e;
  }
  return h + l;
}

template <class Acc>
__device__ __forceinline__ void finish_normal(int cnt, const Acc& acc, const float* __restrict__ prior, int oi,
                                              float* __restrict__ out) {
  double c[6];
  if (cnt >= 3) acc.cov(cnt, c);
  else {
    c[0] = 1; c[1] = 0; c[2] = 0; c[3] = 1; c[4] = 0; c[5] = 0;
  }
  double nv[3];
  fast_eigen3x3(c, nv);
  if (ddot(nv, nv) == 0.0) {
    if (prior) {
      nv[0] = prior[3 * oi]; nv[1] = prior[3 * oi + 1]; nv[2] = prior[3 * oi + 2];
    } else {
      nv[0] = 0; nv[1] = 0; nv[2] = 1;
    }
  }
  if (prior) {
    double pr[3] = {prior[3 * oi], prior[3 * oi + 1], prior[3 * oi + 2]};
    if (ddot(nv, pr) < 0.0) {
      nv[0] = -nv[0]; nv[1] = -nv[1]; nv[2] = -nv[2];
    }
  }
  out[3 * oi] = (float)nv[0];
  out[3 * oi + 1] = (float)nv[1];
  out[3 * oi + 2] = (float)nv[2];
}

template <int K>
__device__ __forceinline__ void knn_normal_query(const GridView& g, const float* __restrict__ xyz, int kneed, int hybrid,
                                 double radius, const float* __restrict__ prior, float* __restrict__ out, int64_t s);

template <int K>
__global__ void __launch_bounds__(kBlock) k_normals_knn(GridView g, const float* __restrict__ xyz, int kneed,
                                                        int hybrid, double radius, const float* __restrict__ prior,
                                                        float* __restrict__ out, const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ list_len) {
  const int64_t lim = list ? (int64_t)*list_len : g.n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < lim; t += (int64_t)gridDim.x * blockDim.x)
    knn_normal_query<K>(g, xyz, kneed, hybrid, radius, prior, out, list ? list[t] : t);
}

template <int K>
__device__ __forceinline__ void knn_normal_query(const GridView& g, const float* __restrict__ xyz, int kneed, int hybrid,
                                 double radius, const float* __restrict__ prior, float* __restrict__ out, int64_t s) {
  const float4 q = g.pts[s];
  const int oi = __float_as_int(q.w);
  double bd[K];
  int bi[K];
  const int cnt = knn_search_dev<K>(g, q.x, q.y, q.z, kneed, hybrid != 0, radius, bd, bi);
  MomAccDD acc;
  acc.zero();
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (j < cnt) {
      const int id = bi[j];
      if (g.nbr && j < kneed) g.nbr[(int64_t)oi * kneed + j] = id;
      if (g.kd2 && j == cnt - 1) g.kd2[oi] = (float)(bd[j] * (1.0 + 1e-6));
      acc.add((double)xyz[3 * id], (double)xyz[3 * id + 1], (double)xyz[3 * id + 2]);
    }
  finish_normal(cnt, acc, prior, oi, out);
}


// ---------------------------------------------------------------------------
// KNN normals, histogram-select form (the default KNN path).
//
// Per query, over the candidates of a neighbourhood inside which every point
// closer than R has been scanned (R = S h + m - slack):
//   count   float32 d^2 of every candidate; the ones inside R are counted
//           into 16 bins uniform in d^2 (packed counters in registers); the
//           wave form grows S until >= k lie inside R;
//   locate  the bin b* holding the k-th distance -> [L, U); while b* holds
//           more than kRefineAt points, re-bin [L, U) into 16 sub-bins
//           (another scan, at most kMaxRefine times);
//   select  rescan: d^2 < L(1-2e) is certainly among the k nearest (appended
//           to an LDS list), d^2 in the band [L(1-2e), U(1+2e)) is a boundary
//           candidate (LDS list), the rest is certainly out — e = 2^-20 bounds
//           the float32 distance error relative to float64;
//   finish  (finish_selection) the (k - #certain) nearest band candidates by
//           exact float64 (d^2, original index) — the oracle's / nanoflann's
//           order — then a check that every certain member precedes every
//           unselected band member in that order, then Open3D's float64 raw
//           moments over the k selected and FastEigen3x3.
// No per-candidate sorted insertion: cost is ~2 scans of the neighbourhood in
// float32 plus O(k) float64 work.  Queries a form cannot settle are appended
// to a list for the next form (LDS tile, lane per query -> wave per query ->
// register top-k).
constexpr int kHistBins = 16;
constexpr int kBndCap = 16;
constexpr int kRefineAt = kBndCap - 2;  // tiles: refine only where the band would overflow
constexpr int kMaxRefine = 2;
constexpr float kRelEps = 9.5367431640625e-07f;  // 2^-20

template <bool W8>
struct RegHist {
  static constexpr int kWords = W8 ? 4 : 8;
  static constexpr int kPer = W8 ? 4 : 2;  // bins per word
  static constexpr int kBits = W8 ? 8 : 16;
  static constexpr int kMaxTotal = W8 ? 255 : 65535;
  uint32_t h[kWords];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < kWords; ++i) h[i] = 0u;
  }
  __device__ __forceinline__ void add(int b) {
    const uint32_t inc = 1u << ((b % kPer) * kBits);
    const int w = b / kPer;
#pragma unroll
    for (int i = 0; i < kWords; ++i) h[i] += (w == i) ? inc : 0u;
  }
  __device__ __forceinline__ int count(int b) const {  // b a compile-time constant after unrolling
    return (int)((h[b / kPer] >> ((b % kPer) * kBits)) & ((1u << kBits) - 1u));
  }
};


// Locate the bin of the k-th distance in a histogram over [lo, hi) with
// `below` points known below lo.  -> bin edges [*L, *U), *cum = points in the
// bins before it, *cb = points in it; false when no bin reaches k.
template <class H, int NB = kHistBins>
__device__ __forceinline__ bool hist_locate(const H& hist, int kneed, int below, float lo, float hi,
                                            float* L, float* U, int* cum, int* cb, int* bin = nullptr) {
  const float bw = (hi - lo) / (float)NB;
  int bstar = -1, c0 = 0, cn = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int c = hist.count(b);
    if (bstar < 0) {
      if (below + c0 + c >= kneed) {
        bstar = b;
        cn = c;
      } else {
        c0 += c;
      }
    }
  }
  *cum = c0;
  *cb = cn;
  if (bin) *bin = bstar;
  *L = lo + (float)bstar * bw;
  *U = (bstar == NB - 1) ? hi : lo + (float)(bstar + 1) * bw;
  return bstar >= 0;
}

// Exact completion of a tile selection (see above).  lst[0..n) holds every
// candidate with f32 d^2 < Up (LDS slots understood by `fetch`).
//   1. one pass over the list, four entries per step with all their LDS loads
//      issued first: certain entries (d^2 < Lm) go straight into the float64
//      moments, band entries are compacted to the front of the list (the
//      write position never passes the read position);
//   2. the band (<= kBndCap entries) in registers with its float32 d^2: the
//      (k - #certain) nearest are picked by repeated minimum and added;
//   3. the picked and unpicked band keys, and the certain keys and the
//      unpicked band keys, must be separated by more than the float32 error
//      (2^-20 relative each side): then the float64 (d^2, index) order — the
//      oracle's / nanoflann's — selects the same set.
// A band that overflows or a separation within rounding (ties included)
// hands the query on (false) to the exact wave form.  Writes the normal of
// original point `oi`.
template <int KMAX, class Acc = MomAcc, class T, class Fetch, class Ident>
__device__ __forceinline__ bool finish_selection(const float4 q, int kneed, int n, float Lm, float U, T (*lst)[64],
                                                 int lane, Fetch&& fetch, const float* __restrict__ prior, int oi,
                                                 float* __restrict__ out, int32_t* __restrict__ nbr, Ident&& ident,
                                                 float* __restrict__ kd2, bool skip_eigen = false) {
  Acc acc;
  acc.zero();
  acc.init(q, U * (1.0f + 2.0f * kRelEps), kneed);  // every member lies below the list bound
  int nsel = 0, nb = 0, nU = 0;
  float cmax = 0.0f;  // largest certain key
  int32_t* const nrow = nbr ? nbr + (int64_t)oi * kneed : nullptr;  // test hook
  const float Ub = U * (1.0f + 2.0f * kRelEps);  // the list's bound; entries past it (a wider list) are skipped
  for (int j = 0; j < n; j += 4) {
    int p[4];
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) p[u] = (int)lst[min(j + u, n - 1)][lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = fetch(p[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (j + u < n) {
        const float d2f = dist2_f32(q, v[u].x, v[u].y, v[u].z);  // the scan's value, bit for bit
        nU += d2f < U ? 1 : 0;
        if (d2f < Lm) {
          if (nrow && nsel < kneed) nrow[nsel] = ident(p[u]);
          cmax = fmaxf(cmax, d2f);
          ++nsel;
          acc.add((double)v[u].x, (double)v[u].y, (double)v[u].z);
        } else if (d2f < Ub) {
          lst[min(nb, kBndCap)][lane] = (T)p[u];
          ++nb;
        }
      }
    }
  }
  // nU >= k: the k nearest lie clearly below Up, so nothing past the band can displace them
  if (nsel > kneed || nb > kBndCap || n < kneed || nU < kneed) return false;
  const int need = kneed - nsel;
  float bk[kBndCap];
  int bs[kBndCap];
#pragma unroll
  for (int i = 0; i < kBndCap; ++i) {
    bk[i] = INFINITY;
    bs[i] = 0;
    if (i < nb) {
      bs[i] = (int)lst[i][lane];
      const float4 v = fetch(bs[i]);
      bk[i] = dist2_f32(q, v.x, v.y, v.z);
    }
  }
  uint32_t picked = 0;
  float kmax = -1.0f;
  for (int t = 0; t < need; ++t) {
    float best = INFINITY;
    int bi = 0;
#pragma unroll
    for (int i = 0; i < kBndCap; ++i)
      if (!((picked >> i) & 1u) && bk[i] < best) {
        best = bk[i];
        bi = i;
      }
    picked |= 1u << bi;
    kmax = best;
  }
  float umin = INFINITY;
  int nput = nsel;
#pragma unroll
  for (int i = 0; i < kBndCap; ++i) {
    if (i < nb) {
      if ((picked >> i) & 1u) {
        const float4 v = fetch(bs[i]);
        if (nrow) nrow[nput++] = ident(bs[i]);
        acc.add((double)v.x, (double)v.y, (double)v.z);
      } else {
        umin = fminf(umin, bk[i]);
      }
    }
  }
  if (need < nb) {
    const float sep = 1.0f - 4.0f * kRelEps;
    if (need > 0 && !(kmax < umin * sep)) return false;
    if (nsel > 0 && !(Lm < umin * sep)) return false;
  }
  if (kd2) kd2[oi] = fmaxf(cmax, need > 0 ? kmax : 0.0f) * (1.0f + 4.0f * kRelEps);
  if (skip_eigen) {  // profiling only (O3DX_TILE_DEBUG=4)
    out[3 * oi] = (float)(acc.m[3] + acc.m[5] + acc.m[8]);
    return true;
  }
  finish_normal(kneed, acc, prior, oi, out);
  return true;
}

// finish_selection for the voxel-table kernel, whose list comes in two parts:
// rows [0, ns) hold the candidates of the bins at least two below the k-th
// one (d^2 < L (1 - 2 eps) by construction: certain members, no distance
// needed), rows [ns, ns + nc) those of the two bins below U (classified by
// their f32 d^2 as finish_selection does).  The band's (k - #certain) nearest
// are picked by rank (lower position first among equal keys, as the repeated
// minimum would), over the wave's longest band only.
template <int KMAX, class Fetch, class Ident>
__device__ __forceinline__ bool stile_finish(const float4 q, int kneed, int ns, int nc, float L, float U,
                                             uint16_t (*lst)[64], int lane, Fetch&& fetch,
                                             const float* __restrict__ prior, int oi, float* __restrict__ out,
                                             int32_t* __restrict__ nbr, Ident&& ident, float* __restrict__ kd2,
                                             bool skip_eigen) {
  MomAcc acc;
  acc.zero();
  int32_t* const nrow = nbr ? nbr + (int64_t)oi * kneed : nullptr;  // test hook
  for (int j = 0; j < ns; j += 4) {
    int p[4];
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) p[u] = (int)lst[min(j + u, ns - 1)][lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = fetch(p[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (j + u < ns) {
        if (nrow) nrow[j + u] = ident(p[u]);
        acc.add((double)v[u].x, (double)v[u].y, (double)v[u].z);
      }
    }
  }
  const int n = ns + nc;
  int nsel = ns, nb = 0, nU = ns;
  float cmax = ns > 0 ? L : 0.0f;  // a bound of the certain keys
  const float Lm = L * (1.0f - 2.0f * kRelEps), Ub = U * (1.0f + 2.0f * kRelEps);
  for (int j = ns; j < n; j += 4) {
    int p[4];
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) p[u] = (int)lst[min(j + u, n - 1)][lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = fetch(p[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (j + u < n) {
        const float d2f = dist2_f32(q, v[u].x, v[u].y, v[u].z);  // the scan's value, bit for bit
        nU += d2f < U ? 1 : 0;
        if (d2f < Lm) {
          if (nrow && nsel < kneed) nrow[nsel] = ident(p[u]);
          cmax = fmaxf(cmax, d2f);
          ++nsel;
          acc.add((double)v[u].x, (double)v[u].y, (double)v[u].z);
        } else if (d2f < Ub) {
          lst[min(nb, kBndCap)][lane] = (uint16_t)p[u];  // rows already read
          ++nb;
        }
      }
    }
  }
  if (nsel > kneed || nb > kBndCap || n < kneed || nU < kneed) return false;
  const int need = kneed - nsel;
  // the longest band of the lanes here (ballots see only the active lanes; a
  // shuffle would read the registers of lanes that left the kernel early):
  // its bits from the top, nb <= kBndCap < 32
  int nbm = 0;
#pragma unroll
  for (int bit = 4; bit >= 0; --bit)
    if (__ballot(nb >= (nbm | (1 << bit)))) nbm |= 1 << bit;
  float bk[kBndCap];
  int bs[kBndCap];
#pragma unroll
  for (int i = 0; i < kBndCap; ++i) {
    bk[i] = INFINITY;
    bs[i] = 0;
    if (i < nbm && i < nb) {
      bs[i] = (int)lst[i][lane];
      const float4 v = fetch(bs[i]);
      bk[i] = dist2_f32(q, v.x, v.y, v.z);
    }
  }
  float kmax = -1.0f, umin = INFINITY;
  int nput = nsel;
#pragma unroll
  for (int i = 0; i < kBndCap; ++i) {
    if (i < nbm) {
      int rank = 0;
#pragma unroll
      for (int j = 0; j < kBndCap; ++j)
        if (j != i && j < nbm) rank += (j < i ? bk[j] <= bk[i] : bk[j] < bk[i]) ? 1 : 0;
      if (i < nb) {
        if (rank < need) {
          kmax = fmaxf(kmax, bk[i]);
          const float4 v = fetch(bs[i]);
          if (nrow) nrow[nput++] = ident(bs[i]);
          acc.add((double)v.x, (double)v.y, (double)v.z);
        } else {
          umin = fminf(umin, bk[i]);
        }
      }
    }
  }
  if (need < nb) {
    const float sep = 1.0f - 4.0f * kRelEps;
    if (need > 0 && !(kmax < umin * sep)) return false;
    if (nsel > 0 && !(Lm < umin * sep)) return false;
  }
  if (kd2) kd2[oi] = fmaxf(cmax, need > 0 ? kmax : 0.0f) * (1.0f + 4.0f * kRelEps);
  if (skip_eigen) {  // profiling only (O3DX_TILE_DEBUG=4)
    out[3 * oi] = (float)(acc.m[3] + acc.m[5] + acc.m[8]);
    return true;
  }
  finish_normal(kneed, acc, prior, oi, out);
  return true;
}

// The float64 tiles' completion (GridView::pts64: a float64 cloud whose tile
// distances are float32 FRAME distances, within g.d64 of the exact ones).
// lst[0..n) holds every candidate with frame d^2 < Ub; entries with frame d^2
// < Lm are certain members, the rest are the band.  The band's (k - #certain)
// nearest are picked by the EXACT float64 (d^2, original index) order; then
// all k members are sorted by it (a bitonic network over 32 registers) and
// summed in that order with separate float64 products and sums — nanoflann's
// result order and Open3D's ComputeCovariance arithmetic, for the same bits
// as the float64 lane-per-query form (k_normals_knn64).
struct Key64 {
  double d;
  int g;  // sorted grid position: the exact coordinates (pts64[g], w = the original index)
};
// (d^2, original index) order; the index is read only on an exact d^2 tie
__device__ __forceinline__ bool key_less(const Key64& a, const Key64& b, const double4* __restrict__ pts64) {
  if (a.d != b.d) return a.d < b.d;
  return a.g != b.g && pts64[a.g].w < pts64[b.g].w;
}
template <int I, int J, bool UP>
__device__ __forceinline__ void key_ce(Key64 (&k)[32], const double4* __restrict__ pts64) {
  const bool sw = UP ? key_less(k[J], k[I], pts64) : key_less(k[I], k[J], pts64);
  const Key64 a = k[I], b = k[J];
  k[I].d = sw ? b.d : a.d;
  k[I].g = sw ? b.g : a.g;
  k[J].d = sw ? a.d : b.d;
  k[J].g = sw ? a.g : b.g;
}
// bitonic sort of 32 keys, ascending (compile-time indices throughout)
template <int SZ, int ST, int I>
__device__ __forceinline__ void key_stage(Key64 (&k)[32], const double4* __restrict__ pts64) {
  if constexpr (I < 32) {
    constexpr int J = I ^ ST;
    if constexpr (J > I) key_ce<I, J, (I & SZ) == 0>(k, pts64);
    key_stage<SZ, ST, I + 1>(k, pts64);
  }
}
template <int SZ, int ST>
__device__ __forceinline__ void key_merge(Key64 (&k)[32], const double4* __restrict__ pts64) {
  if constexpr (ST > 0) {
    key_stage<SZ, ST, 0>(k, pts64);
    key_merge<SZ, ST / 2>(k, pts64);
  }
}
template <int SZ>
__device__ __forceinline__ void key_sort(Key64 (&k)[32], const double4* __restrict__ pts64) {
  if constexpr (SZ <= 32) {
    key_merge<SZ, SZ / 2>(k, pts64);
    key_sort<SZ * 2>(k, pts64);
  }
}

__device__ __forceinline__ Key64 key64_of(const double4* __restrict__ pts64, double qx, double qy, double qz,
                                          const int32_t* tp, int p) {
  const int g = tp[p];
  return Key64{dist2_d4(qx, qy, qz, pts64[g]), g};
}

// (the grid's members by value: a GridView reference would put the kernel
// argument in scratch)
__device__ __forceinline__ bool finish_selection64(const double4* __restrict__ pts64, const double* __restrict__ xyz,
                                                   int32_t* __restrict__ nbr, float* __restrict__ kd2, double qx,
                                                   double qy, double qz,
                                                   const float4 q, int kneed, int n, float Lm, float U, float Ub,
                                                   uint16_t (*lst)[64], uint16_t (*band)[64], int lane,
                                                   const float* tx, const float* ty, const float* tz,
                                                   const int32_t* tp, const float* __restrict__ prior, int oi,
                                                   float* __restrict__ out) {
  // 1. certain members compacted to the front of the list, the band apart
  int nsel = 0, nb = 0, nU = 0;
  for (int j = 0; j < n; ++j) {
    const int p = (int)lst[j][lane];
    const float d2f = dist2_f32(q, tx[p], ty[p], tz[p]);
    nU += d2f < U ? 1 : 0;
    if (d2f < Lm) {
      lst[nsel][lane] = (uint16_t)p;  // (the write position never passes the read position)
      ++nsel;
    } else if (d2f < Ub) {
      band[min(nb, kBndCap)][lane] = (uint16_t)p;
      ++nb;
    }
  }
  // nU >= k: the k-th nearest lies within sqrt(U) + d64, so all k nearest are listed
  if (nsel > kneed || nb > kBndCap || nsel + nb < kneed || nU < kneed) return false;
  const int need = kneed - nsel;
  // 2. the band's `need` nearest by the exact order, appended
  Key64 bk[kBndCap];
#pragma unroll
  for (int i = 0; i < kBndCap; ++i) {
    bk[i] = Key64{INFINITY, -1};
    if (i < nb) bk[i] = key64_of(pts64, qx, qy, qz, tp, (int)band[i][lane]);
  }
  uint32_t picked = 0;
  for (int t = 0; t < need; ++t) {  // repeated minimum (register indices stay compile-time)
    Key64 best{INFINITY, -1};
    int bi = 0;
#pragma unroll
    for (int i = 0; i < kBndCap; ++i)
      if (!((picked >> i) & 1u) && (best.g < 0 || key_less(bk[i], best, pts64))) {
        best = bk[i];
        bi = i;
      }
    picked |= 1u << bi;
    lst[nsel + t][lane] = band[bi][lane];
  }
  // 3. the k members in the exact order, Open3D's sequential moments
  Key64 kk[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    kk[i] = Key64{INFINITY, 0x7fffffff};  // padding: after every member (INFINITY ties only padding)
    if (i < kneed) kk[i] = key64_of(pts64, qx, qy, qz, tp, (int)lst[i][lane]);
  }
  key_sort<2>(kk, pts64);
  MomAccSeq acc;
  acc.zero();
  int32_t* const nrow = nbr ? nbr + (int64_t)oi * kneed : nullptr;  // test hook
  double dk = 0.0;  // the k-th key (no dynamic index into the register array)
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    if (i < kneed) {
      const double4 v = pts64[kk[i].g];
      if (nrow) nrow[i] = (int)v.w;
      acc.add(v.x, v.y, v.z);
      dk = kk[i].d;
    }
  }
  if (kd2) kd2[oi] = (float)(dk * (1.0 + 1e-6));
  finish_normal(kneed, acc, prior, oi, out);
  return true;
}

// ---------------------------------------------------------------------------
// KNN normals, LDS-tile form (first level of the default KNN path).
// One block = one wave = one chunk of <= 64 consecutive queries in one grid
// row; the 9-row neighbour box is staged into LDS (coalesced, SoA f32), then
// every lane runs the histogram-select steps over LDS-resident candidates
// (shells 0..1 only).  The histogram lives in LDS (in the selection list's
// space, unused until the select scan): 18 packed 16-bit slots per lane —
// 0 below the range, 1..16 the bins, 17 at or above it — word-major [9][64]
// so each lane owns a bank column, updated with ds_add (no dependency on
// the previous update).  Queries the tile cannot settle (fewer than k points
// within the shell-1 radius, the band overflows, the order check fails, or
// a single cell's box does not fit in LDS) are appended to fb_list for the
// wave form.  A chunk whose box does not fit is processed in x-halves.
constexpr int kTileQ = 64;
constexpr int kTilePts = 960;
constexpr int kTileCs = 384;

// Blocks are dealt round-robin over the 8 XCDs (b and b+8 share one, each XCD
// has its own L2): give each XCD a contiguous run of chunks, so the rows a
// chunk stages were mostly staged just before by its neighbours on the same
// XCD.  A bijection on [0, nb).
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int x = b & 7, i = b >> 3, q = nb >> 3, r = nb & 7;
  return x * q + min(x, r) + i;
}

constexpr int kTileSlots = kHistBins + 2;  // below the range, the bins, at or above it

struct TileHist {
  uint32_t h[kTileSlots];
  __device__ __forceinline__ int count(int b) const { return (int)h[b + 1]; }  // b in -1..16
};

typedef float f32x2 __attribute__((ext_vector_type(2)));

// f32 d^2 of two candidates with packed math (v_pk_add / v_pk_mul / v_pk_fma):
// the same operations and roundings as dist2_f32, two lanes of work per op.
__device__ __forceinline__ f32x2 dist2_pair(const float4 q, f32x2 x, f32x2 y, f32x2 z) {
  const f32x2 dx = (f32x2){q.x, q.x} - x, dy = (f32x2){q.y, q.y} - y, dz = (f32x2){q.z, q.z} - z;
  return __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
}

// Row r (0..8) of the 3x3 (y,z) rows around (cy,cz), clipped to the box and
// to x in [cx-1, cx+1], then trimmed to the cells whose box (grown by the
// rounding slack) comes closer to q than sqrt(bound): LDS slots [*a, *e).
// A trimmed cell holds no point with f32 d^2 below bound, so no scan that
// only counts / selects d^2 < bound can miss anything.
__device__ __forceinline__ void tile_row(const GridView& g, const TileBox& b, const int32_t* ccs, const float4 q,
                                         int cx, int cy, int cz, int r, float bound, int* a, int* e) {
  const int z = cz + r / 3 - 1, y = cy + r % 3 - 1;
  *a = *e = 0;
  if (z < b.z0 || z > b.z1 || y < b.y0 || y > b.y1) return;
  const float lim = bound * (1.0f + 1e-5f);
  const float y0 = g.oy + (float)y * g.h, z0 = g.oz + (float)z * g.h;
  const float gy = fmaxf(fmaxf(y0 - q.y, q.y - (y0 + g.h)) - g.slack, 0.0f);
  const float gz = fmaxf(fmaxf(z0 - q.z, q.z - (z0 + g.h)) - g.slack, 0.0f);
  const float dyz = gy * gy + gz * gz;
  if (dyz > lim) return;
  int xa = max(cx - 1, b.x0), xb = min(cx + 1, b.x1);
  if (xa < cx) {
    const float gx = fmaxf(q.x - (g.ox + (float)cx * g.h) - g.slack, 0.0f);
    if (dyz + gx * gx > lim) xa = cx;
  }
  if (xb > cx) {
    const float gx = fmaxf((g.ox + (float)(cx + 1) * g.h) - q.x - g.slack, 0.0f);
    if (dyz + gx * gx > lim) xb = cx;
  }
  const int w = b.nxr + 1;
  const int k = (y - b.y0) + b.nyr * (z - b.z0);
  *a = ccs[k * w + xa - b.x0];
  *e = ccs[k * w + xb - b.x0 + 1];
}

// Candidates of the query's 27-cell cube from the LDS tile, four at a time
// (LDS loads issued before use, distances two at a time in packed f32).
#define O3DX_TILE_SCAN(BOUND, BODY)                                        \
  for (int r_ = 0; r_ < 9; ++r_) {                                         \
    int a_, e_;                                                            \
    tile_row(g, box, ccs, q, cx, cy, cz, r_, (BOUND), &a_, &e_);           \
    int p_ = a_;                                                           \
    for (; p_ + 4 <= e_; p_ += 4) {                                        \
      const f32x2 xa_ = {tx[p_], tx[p_ + 1]}, xb_ = {tx[p_ + 2], tx[p_ + 3]}; \
      const f32x2 ya_ = {ty[p_], ty[p_ + 1]}, yb_ = {ty[p_ + 2], ty[p_ + 3]}; \
      const f32x2 za_ = {tz[p_], tz[p_ + 1]}, zb_ = {tz[p_ + 2], tz[p_ + 3]}; \
      const f32x2 da_ = dist2_pair(q, xa_, ya_, za_);                      \
      const f32x2 db_ = dist2_pair(q, xb_, yb_, zb_);                      \
      const float ds_[4] = {da_.x, da_.y, db_.x, db_.y};                   \
      _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_) {                   \
        const int pp = p_ + u_;                                            \
        (void)pp;                                                          \
        const float d2 = ds_[u_];                                          \
        BODY                                                               \
      }                                                                    \
    }                                                                      \
    for (; p_ < e_; ++p_) {                                                \
      const int pp = p_;                                                   \
      (void)pp;                                                            \
      const float d2 = dist2_f32(q, tx[p_], ty[p_], tz[p_]);               \
      BODY                                                                 \
    }                                                                      \
  }

// Histogram of the cube's candidates over [LO, HI = LO + 16/SC) into the LDS
// counters `hw` (slot-major [18][64]: each lane owns a bank column; ds_add,
// no return), then into registers `th`; cells entirely beyond HI skipped.
#define O3DX_TILE_HIST(LO, SC, HI)                                                          \
  {                                                                                         \
    _Pragma("unroll") for (int i_ = 0; i_ < kTileSlots; ++i_) hw[i_ * 64 + lane] = 0u;     \
    const float off_ = -(LO) * (SC);                                                        \
    O3DX_TILE_HIST_SCAN((HI), (SC), off_)                                                   \
    _Pragma("unroll") for (int i_ = 0; i_ < kTileSlots; ++i_) th.h[i_] = hw[i_ * 64 + lane]; \
  }
#define O3DX_TILE_HIST_SCAN(HI, SC, OFF)                                                    \
  O3DX_TILE_SCAN(HI, {                                                                      \
    const int ix_ = (int)fminf(fmaxf(fmaf(d2, (SC), (OFF)), -1.0f), 16.0f);                 \
    atomicAdd(&hw[(ix_ + 1) * 64 + lane], 1u);                                              \
  })

// F64: a float64 cloud's grid (GridView::pts64, frame coordinates in pts):
// the same scans on the frame, widened by the frame error g.d64, and the
// exact completion finish_selection64 (KMAX 32).
template <int KMAX, class TAcc = MomAccA, bool F64 = false>
__global__ void __launch_bounds__(kTileQ) __attribute__((amdgpu_waves_per_eu(2))) k_normals_knn_tile(GridView g, const int32_t* __restrict__ chunk_starts,
                                                             int kneed, const float* __restrict__ prior,
                                                             float* __restrict__ out, int32_t* __restrict__ fb_list,
                                                             int32_t* __restrict__ fb_len, int dbg) {
  static_assert(kTileQ == 64, "one wave per tile");
  static_assert(!F64 || KMAX == 32, "float64 tiles sort 32 keys");
  __shared__ float tx[kTilePts], ty[kTilePts], tz[kTilePts];
  __shared__ int32_t tp[F64 ? kTilePts : 1];              // float64: the slots' global positions
  __shared__ uint16_t band64[F64 ? kBndCap + 1 : 1][64];  // float64: the band apart from the list
  __shared__ int32_t ccs[kTileCs];
  __shared__ int32_t rows[kMaxTileRows + 1];
  __shared__ int32_t rst[kMaxTileRows];
  // the candidate list (u16 [KMAX + band + 1][64]) and the histogram counters
  // (u32 [18][64]) share one LDS buffer: the histogram is dead before the list
  constexpr int kListMax = KMAX + kBndCap;      // more entries than this: hand the query on
  constexpr int kListCap = kListMax + 4;        // room for one unconditional 4-candidate store
  constexpr int kListWords = (kListCap * kTileQ * 2 + 3) / 4;
  constexpr int kHistWords = kTileSlots * kTileQ;
  __shared__ uint32_t selbuf[kListWords > kHistWords ? kListWords : kHistWords];
  uint16_t(*lst)[kTileQ] = reinterpret_cast<uint16_t(*)[kTileQ]>(selbuf);
  const int lane = threadIdx.x;
  // the launch covers an upper bound of the chunk count; the real count sits
  // after the list, and the XCD-contiguous mapping spans the real chunks only
  const int nreal = chunk_starts[gridDim.x + 1];
  if ((int)blockIdx.x >= nreal) return;
  const int c = xcd_block(blockIdx.x, nreal);
  const int q0 = chunk_starts[c], q1 = chunk_starts[c + 1];
  const int64_t s = (int64_t)q0 + lane;
  bool active = s < q1;
  // the chunk lies in one z slab and spans a few y rows (each sorted by x)
  const float4 q = g.pts[active ? s : (int64_t)q0];
  int cx, cy, cz;
  grid_cell(g, q.x, q.y, q.z, cx, cy, cz);
  const int qw = __float_as_int(q.w);
  if (g.outer) {
    active = active && qw >= 0;  // a nested grid's candidate-only point
  } else if (g.skip_cells) {     // the queries near dense cells are the nested grid's
    active = active && !g.skip_cells[cell_index(g, cx, cy, cz)];
  }
  int az;
  {
    const float4 f = g.pts[q0];
    int fx, fy;
    grid_cell(g, f.x, f.y, f.z, fx, fy, az);
  }
  const int ay0 = wave_min(active ? cy : INT_MAX), ay1 = wave_max(active ? cy : INT_MIN);
  bool fb = active && cz != az;
  bool todo = active && !fb;
  // Parts: x-cell ranges [lowest unprocessed cx, highest cx] of the chunk's
  // lanes, left to right.  A part whose box does not fit in LDS is halved
  // (down to one cell) before it is staged.
  for (;;) {
    const int x_lo = wave_min(todo ? cx : INT_MAX);
    if (x_lo == INT_MAX) break;
    int x_hi = wave_max(todo ? cx : INT_MIN), staged;
    TileBox box;
    for (;;) {
      box.x0 = max(x_lo - 1, 0);
      box.x1 = min(x_hi + 1, g.nx - 1);
      box.y0 = max(ay0 - 1, 0);
      box.y1 = min(ay1 + 1, g.ny - 1);
      box.z0 = max(az - 1, 0);
      box.z1 = min(az + 1, g.nz - 1);
      box.nxr = box.x1 - box.x0 + 1;
      box.nyr = box.y1 - box.y0 + 1;
      staged = stage_tile<kTileQ, kTilePts>(g, box, tx, ty, tz, ccs, kTileCs, rows, rst, F64 ? tp : nullptr);
      if (staged >= 0 || x_hi == x_lo) break;
      __syncthreads();
      x_hi = x_lo + (x_hi - x_lo) / 2;
    }
    const bool mine = todo && cx >= x_lo && cx <= x_hi;
    if (mine) todo = false;
    if (mine && dbg != 1) {
      fb = staged < 0;
      if (fb && g.stats) atomicAdd(&g.stats[6], 1ull);
      if (!fb) {
        const double reach = cube_reach(g, q.x, q.y, q.z, cx, cy, cz, 1);
        double R = (reach == INFINITY) ? (double)(g.nx + g.ny + g.nz) * g.h : reach - g.slack;
        R = fmin(R, outer_reach(g, q.x, q.y, q.z));
        // float64: the k nearest by exact distance lie within frame distance
        // sqrt(U) + 2 d64 of the frame query, which must stay inside R
        if (F64) R -= 2.0 * (double)g.d64;
        const float R2 = (R > 0.0) ? (float)(R * R) * (1.0f - (F64 ? 16.0f : 4.0f) * kRelEps) : 0.0f;
        uint32_t* hw = selbuf;
        TileHist th;
        O3DX_TILE_HIST(0.0f, (float)kHistBins / fmaxf(R2, 1e-30f), R2)
        int total = 0;
#pragma unroll
        for (int b = 0; b < kHistBins; ++b) total += th.count(b);
        fb = total < kneed;
        if (fb && g.stats) atomicAdd(&g.stats[7], 1ull);
        float lo = 0.f, hi = R2, L = 0.f, U = 0.f;
        for (int lvl = 0; !fb; ++lvl) {
          int cum, cb;
          if (!hist_locate(th, kneed, th.count(-1), lo, hi, &L, &U, &cum, &cb)) {
            fb = true;
            break;
          }
          if (cb <= kRefineAt || lvl == kMaxRefine || !(U > L)) break;
          lo = L;
          hi = U;
          O3DX_TILE_HIST(lo, (float)kHistBins / (hi - lo), hi)
        }
        if (!fb && dbg != 2) {
          float Lm = L * (1.0f - 2.0f * kRelEps), Up = U * (1.0f + 2.0f * kRelEps);
          if constexpr (F64) {  // frame distances: certain below sqrt(L) - 2 d64, listed below sqrt(U) + 2 d64
            const float e2 = 2.0f * g.d64, sl = sqrtf(L) * (1.0f - 2.0f * kRelEps) - e2;
            Lm = sl > 0.0f ? sl * sl * (1.0f - 4.0f * kRelEps) : -1.0f;
            const float su = sqrtf(U) * (1.0f + 2.0f * kRelEps) + e2;
            Up = su * su * (1.0f + 4.0f * kRelEps);
          }
          // branch-free append of every candidate below Up: candidate u of a
          // group of four is written to slot n + (#accepted before u), so the
          // accepted ones end up contiguous and a rejected one is overwritten
          // by the next accepted (or by the next group); one clamp per group
          int n = 0;
          for (int r_ = 0; r_ < 9; ++r_) {
            int a_, e_;
            tile_row(g, box, ccs, q, cx, cy, cz, r_, Up, &a_, &e_);
            int p_ = a_;
            for (; p_ + 4 <= e_; p_ += 4) {
              const f32x2 da_ = dist2_pair(q, (f32x2){tx[p_], tx[p_ + 1]}, (f32x2){ty[p_], ty[p_ + 1]},
                                           (f32x2){tz[p_], tz[p_ + 1]});
              const f32x2 db_ = dist2_pair(q, (f32x2){tx[p_ + 2], tx[p_ + 3]}, (f32x2){ty[p_ + 2], ty[p_ + 3]},
                                           (f32x2){tz[p_ + 2], tz[p_ + 3]});
              const int a0 = da_.x < Up, a1 = da_.y < Up, a2 = db_.x < Up, a3 = db_.y < Up;
              uint16_t* base = &lst[min(n, kListMax)][lane];
              base[0] = (uint16_t)p_;
              base[a0 * kTileQ] = (uint16_t)(p_ + 1);
              base[(a0 + a1) * kTileQ] = (uint16_t)(p_ + 2);
              base[(a0 + a1 + a2) * kTileQ] = (uint16_t)(p_ + 3);
              n += a0 + a1 + a2 + a3;
            }
            for (; p_ < e_; ++p_) {
              lst[min(n, kListMax)][lane] = (uint16_t)p_;
              n += dist2_f32(q, tx[p_], ty[p_], tz[p_]) < Up ? 1 : 0;
            }
          }
          if (dbg == 3) {
            if (n == 12345) out[0] = 0.f;  // keep the scan alive
          } else if constexpr (F64) {
            const double4 q64 = g.pts64[s];
            fb = n > kListMax || !finish_selection64(g.pts64, g.xyz64, g.nbr, g.kd2, q64.x, q64.y, q64.z, q, kneed, n, Lm, U,
                                                     Up, lst, band64, lane, tx, ty, tz, tp, prior, out_row(g, qw),
                                                     out);
          } else
          fb = n > kListMax ||
               !finish_selection<KMAX, TAcc>(
                   q, kneed, n, Lm, U, lst, lane, [&](int p) { return make_float4(tx[p], ty[p], tz[p], 0.f); },
                   prior, out_row(g, qw), out, g.nbr,
                   [&](int p) { return out_row(g, __float_as_int(g.pts[tile_global_pos(rows, rst, p)].w)); }, g.kd2,
                   dbg == 4);
        }
      }
    }
    __syncthreads();  // the next part restages the LDS tile
  }
  if (fb) {
    if (g.stats) atomicAdd(&g.stats[4], 1ull);
    const int at = atomicAdd(fb_len, 1);
    fb_list[at] = g.outer ? qw : (int32_t)s;  // the outer grid's wave form takes a nested grid's hand-offs
  }
}
#undef O3DX_TILE_SCAN
#undef O3DX_TILE_HIST
#undef O3DX_TILE_HIST_SCAN

// ---------------------------------------------------------------------------
// KNN normals straight off a dense voxel table (the voxel_down_sample ->
// estimate_normals hand-over, o3dx_estimate_normals_voxel), used when the
// representatives fill their voxels (<= 1 rep per voxel by construction; most
// voxels occupied — any volumetric cloud after down-sampling).  No search
// grid is built: the voxel table is the grid, at voxel granularity.
//
// One workgroup = 2 x 2 waves, each wave a block of 4^3 voxels (lane = voxel
// = query).  The workgroup's box (4 x 8 x 8 voxels + a 3-voxel margin) is
// staged once from the table into LDS ((x, y) interleaved float2 + z apart;
// empty voxel: +inf, never inside any bound).  Every lane scans a fixed
// stencil around its own voxel: the voxels that can hold a point within R
// voxels of a query in the upper half of its voxel along each axis, mirrored
// per axis to the half the lane's query is in.  Row offsets and lengths are
// compile-time constants, so lanes never diverge in the scans.
//   count   R = 2.2 voxels (148 voxels; the k = 30 neighbour of an interior
//           query at one rep per voxel lies within 2.2 for all but ~1e-5 of
//           them): f32 d^2 into 16 LDS bins over [(1.5 voxels)^2, R^2) (the
//           k-th neighbour of a voxelised cloud is never that close in
//           practice: bins where the k-th distances are; a k-th below them
//           hands the query on);
//   locate  the bin holding the k-th distance -> [L, U) (refined <= 2 times);
//   list    rescan with the smallest of the R = 2.1 / 2.2 stencils (136 / 148
//           voxels) that covers the wave's largest U, appending d^2 < U;
//   finish  exact (d^2, index) selection (finish_selection), f64 moments,
//           FastEigen3x3.
// Queries whose k-th neighbour lies beyond R (cloud borders, sparse spots) go
// by voxel index to the wave form and the register top-k over the table.
// (Measured and dropped, DESIGN.md §4.1: a symmetric stencil, a merged
// count+list pass, a list-first form, compact 1-byte lists, 1x1 / 2x3 blocks.)
constexpr int kVB = 4;                     // block edge (voxels)
constexpr int kVM = 3;                     // box margin (the stencil's reach in voxels)
constexpr int kVE = kVB + 2 * kVM;         // box edge (10)
constexpr double kStencilR = 2.2;          // completeness radius of the count stencil (voxels)
constexpr double kListR = 2.1;             // the smaller list stencil (voxels)
constexpr double kHistLo = 1.5;            // the count histogram's lower edge (voxels)
constexpr double kWideR = 2.45;            // the border waves' stencil (voxels)
constexpr int kEdge = 3;                   // border waves: within kEdge voxels of a table face

struct SRow {
  int dy, dz, xa, len;
};

// (dy, dz, x0, len) in the oriented frame (query in [0.49, 1) of its voxel on
// every axis): the voxels within R of any such query (tools/stencil_rows.py)
struct Stencil220 {
  static constexpr SRow rows[] = {
      {-2, -2, -1, 3}, {-1, -2, -2, 5}, {0, -2, -2, 5}, {1, -2, -2, 5}, {2, -2, -1, 4}, {-2, -1, -2, 5},
      {-1, -1, -2, 6}, {0, -1, -2, 6},  {1, -1, -2, 6}, {2, -1, -2, 5}, {3, -1, -1, 3}, {-2, 0, -2, 5},
      {-1, 0, -2, 6},  {0, 0, -2, 6},   {1, 0, -2, 6},  {2, 0, -2, 5},  {3, 0, -1, 3},  {-2, 1, -2, 5},
      {-1, 1, -2, 6},  {0, 1, -2, 6},   {1, 1, -2, 6},  {2, 1, -2, 5},  {3, 1, -1, 3},  {-2, 2, -1, 4},
      {-1, 2, -2, 5},  {0, 2, -2, 5},   {1, 2, -2, 5},  {2, 2, -2, 5},  {-1, 3, -1, 3}, {0, 3, -1, 3},
      {1, 3, -1, 3}};
  static constexpr int N = (int)(sizeof(rows) / sizeof(SRow));
};
struct Stencil245 {  // the waves at the cloud's borders (a wider ball keeps their k nearest in it)
  static constexpr SRow rows[] = {
      {-2, -2, -1, 4}, {-1, -2, -2, 5}, {0, -2, -2, 5}, {1, -2, -2, 5}, {2, -2, -2, 5}, {-2, -1, -2, 5},
      {-1, -1, -2, 6}, {0, -1, -2, 6},  {1, -1, -2, 6}, {2, -1, -2, 6}, {3, -1, -1, 4}, {-2, 0, -2, 5},
      {-1, 0, -2, 6},  {0, 0, -2, 6},   {1, 0, -2, 6},  {2, 0, -2, 6},  {3, 0, -1, 4},  {-2, 1, -2, 5},
      {-1, 1, -2, 6},  {0, 1, -2, 6},   {1, 1, -2, 6},  {2, 1, -2, 6},  {3, 1, -1, 4},  {-2, 2, -2, 5},
      {-1, 2, -2, 6},  {0, 2, -2, 6},   {1, 2, -2, 6},  {2, 2, -2, 6},  {3, 2, -1, 4},  {-1, 3, -1, 4},
      {0, 3, -1, 4},   {1, 3, -1, 4},   {2, 3, -1, 4}};
  static constexpr int N = (int)(sizeof(rows) / sizeof(SRow));
};
struct Stencil210 {
  static constexpr SRow rows[] = {
      {-1, -2, -1, 4}, {0, -2, -1, 4}, {1, -2, -1, 4}, {2, -2, -1, 4}, {-2, -1, -1, 4}, {-1, -1, -2, 5},
      {0, -1, -2, 6},  {1, -1, -2, 6}, {2, -1, -2, 5}, {3, -1, 0, 2},  {-2, 0, -1, 4},  {-1, 0, -2, 6},
      {0, 0, -2, 6},   {1, 0, -2, 6},  {2, 0, -2, 5},  {3, 0, -1, 3},  {-2, 1, -1, 4},  {-1, 1, -2, 6},
      {0, 1, -2, 6},   {1, 1, -2, 6},  {2, 1, -2, 5},  {3, 1, -1, 3},  {-2, 2, -1, 4},  {-1, 2, -2, 5},
      {0, 2, -2, 5},   {1, 2, -2, 5},  {2, 2, -2, 5},  {-1, 3, 0, 2},  {0, 3, -1, 3},   {1, 3, -1, 3}};
  static constexpr int N = (int)(sizeof(rows) / sizeof(SRow));
};

struct DenseVox {
  const float4* __restrict__ vox;  // (x, y, z, bits(row)), row -1 = empty (0xFF fill: NaN coordinates)
  int nx, ny, nz;                  // voxel dims
  int nbx, nby, nbz;               // workgroup blocks
  float ox, oy, oz, vs, inv_vs;
  float rc2;                       // completeness radius^2 of the count stencil (world, f32, shrunk by the slack)
  float rl2;                       // the same for the smaller list stencil
  float rw2;                       // the same for the border waves' wider stencil
  float hlo2;                      // the count histogram's lower edge (world d^2)
  unsigned long long* stats;       // debug counters (o3dx_search_stats) or null
  int32_t* nbr;                    // test hook (o3dx_set_debug_neighbors) or null
  float* kd2;                      // per row an upper bound of the k-th neighbour d^2, or null
};

__device__ __forceinline__ float4 dvox_load(const DenseVox& d, int x, int y, int z) {
  float4 v = make_float4(INFINITY, INFINITY, INFINITY, __int_as_float(-1));
  if (x >= 0 && y >= 0 && z >= 0 && x < d.nx && y < d.ny && z < d.nz) {
    v = d.vox[x + (int64_t)d.nx * (y + (int64_t)d.ny * z)];
    if (__float_as_int(v.w) < 0) v.x = v.y = v.z = INFINITY;
  }
  return v;
}

// Candidates are numbered in stencil order (row by row, ascending slot within
// a row); a scan body receives that number as a compile-time constant.
template <int C>
using IC = std::integral_constant<int, C>;
template <class St>
constexpr int stencil_prefix(int I) {
  int s = 0;
  for (int r = 0; r < I; ++r) s += St::rows[r].len;
  return s;
}
template <class St>
constexpr int stencil_cands() {
  return stencil_prefix<St>(St::N);
}

template <int C0, class F, int... I>
__device__ __forceinline__ void run_bodies(F& f, int st, const float* d2, std::integer_sequence<int, I...>) {
  (f(IC<C0 + I>{}, st + I, d2[I]), ...);
}

// f(IC<candidate>, slot, d2) over the L consecutive slots of a row from st.
// x, y interleaved (each slot's pair by its own ds_read_b64: a volatile load
// is never merged into the 8-cycle ds_read2_b64, MI355X_MICROARCH.md §LDS), z
// apart.  The row's loads are all issued before its first f (whose LDS atomics
// the compiler cannot move reads across).  Distances in plain f32 (v_fma_f32:
// 2 cycles per wave64 instruction, where v_pk_fma_f32 takes 4 and the packing
// costs lane moves; grid.o is built without the SLP vectorizer).
template <int L, int C0, class F>
__device__ __forceinline__ void scan_run(const float2* txy, const float* tz, int st, const float4 q, F& f) {
  float2 a[L];
  float c[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    typedef __attribute__((address_space(3))) const volatile f32x2 lds_vf2;
    const f32x2 v = *(lds_vf2*)(&txy[st + i]);
    a[i] = make_float2(v.x, v.y);
    c[i] = tz[st + i];
  }
  float d2[L];
#pragma unroll
  for (int i = 0; i < L; ++i) d2[i] = dist2_f32(q, a[i].x, a[i].y, c[i]);
  run_bodies<C0>(f, st, d2, std::make_integer_sequence<int, L>{});
}

// a scheduling fence per row keeps the unrolled stencil from hoisting every
// row's loads (register pressure; the other waves hide the LDS latency)
template <class St, int I, class F>
__device__ __forceinline__ void mir_rows(const float2* txy, const float* tz, int qs, int SY, int SZ, bool xpos,
                                         const float4 q, F& f) {
  if constexpr (I < St::N) {
    constexpr SRow r = St::rows[I];
    scan_run<r.len, stencil_prefix<St>(I)>(txy, tz, qs + r.dy * SY + r.dz * SZ + (xpos ? r.xa : -(r.xa + r.len - 1)),
                                           q, f);
    __builtin_amdgcn_sched_barrier(0);
    mir_rows<St, I + 1>(txy, tz, qs, SY, SZ, xpos, q, f);
  }
}

// The lane's stencil: qs = its own slot, SY / SZ = the y / z slot strides
// signed by the orientation, xpos = x orientation.
template <class St, class F>
__device__ __forceinline__ void stencil_scan(const float2* txy, const float* tz, int qs, int SY, int SZ, bool xpos,
                                             const float4 q, F&& f) {
  // the row bases are recomputed per scan (laundered inputs): hoisted and
  // shared across the kernel's scans they would stay live throughout
  asm volatile("" : "+v"(qs), "+v"(SY), "+v"(SZ));
  mir_rows<St, 0>(txy, tz, qs, SY, SZ, xpos, q, f);
}

// The same stencil walk without loads: f(IC<candidate>, slot).
template <int C0, class F, int... I>
__device__ __forceinline__ void walk_bodies(F& f, int st, std::integer_sequence<int, I...>) {
  (f(IC<C0 + I>{}, st + I), ...);
}
template <class St, int I, class F>
__device__ __forceinline__ void walk_rows(int qs, int SY, int SZ, bool xpos, F& f) {
  if constexpr (I < St::N) {
    constexpr SRow r = St::rows[I];
    walk_bodies<stencil_prefix<St>(I)>(f, qs + r.dy * SY + r.dz * SZ + (xpos ? r.xa : -(r.xa + r.len - 1)),
                                       std::make_integer_sequence<int, r.len>{});
    walk_rows<St, I + 1>(qs, SY, SZ, xpos, f);
  }
}

// Block shape: WY x WZ waves, each wave a 4^3 voxel block; the block's box is
// the union (4 x 4WY x 4WZ voxels + the 3-voxel margin), staged once for all
// its waves — 2x2 waves stage 7.7 slots per query instead of 15.6 and fit
// 3 workgroups (12 waves) per CU in LDS.
// The z-plane stride is padded to 16 (mod 32): lanes (x, y, z) and (x, y, z+1)
// of a 32-lane half then read banks 16 apart, and the 32 lanes of a half
// (4 x 4 x 2 voxels) hit 2.3 distinct slots per bank on average under the
// random per-lane mirroring instead of 3.1 (ds_read_b64 / ds_read2_b32: bank =
// slot mod 32; tools/stile_banks.py).
template <int WY, int WZ>
struct StileShape {
  static constexpr int NW = WY * WZ;
  static constexpr int EY = kVB * WY + 2 * kVM, EZ = kVB * WZ + 2 * kVM;
  static constexpr int SY = kVE;
  static constexpr int SZ = kVE * EY + (16 - (kVE * EY) % 32 + 32) % 32;
  static constexpr int NC = kVE * EY * EZ;  // box cells
  static constexpr int CELLS = SZ * EZ;     // LDS slots (padded planes)
};

// The count scan's histogram: 16 slots per lane — 0 below the range, 1..14
// the bins, 15 at or above it — so a candidate's slot fits a nibble.
constexpr int kStileBins = 14;
constexpr int kStileSlots = kStileBins + 2;
struct StileHist {
  uint32_t h[kStileSlots];
  __device__ __forceinline__ int count(int b) const { return (int)h[b + 1]; }  // b in -1..kStileBins
};

// Count scan + list of one lane (stencil St):
//   count   f32 d^2 of the stencil's candidates into the histogram over
//           [lo, hi) (LDS counters, one bank column per lane), each
//           candidate's level-0 slot kept as a nibble in registers (nib);
//   locate  the bin b0 holding the k-th distance -> [L, U) (refined, rarely,
//           by rescans over [L, U));
//   list    the candidates whose level-0 slot is <= b0 + 1, appended to the
//           lane's LDS list without a second distance scan.
// The slot of d^2 is floor(fma(d^2, sc, off)) with an absolute error below
// 2^-18.6 bins, and [lo, hi) sits at >= 1.5 voxels, so every candidate below
// U (1 - 2^-17) has slot <= b0 + 1: the list holds every candidate below the
// finish's band bound U' (1 + 2 eps) for U' = U (1 - 2^-16), passed out as *U.
// Returns false when the lane hands its query on.
template <class St, class LST>
__device__ __forceinline__ bool stile_count_list(const float2* txy, const float* tz, int qs, int SY, int SZ, bool xpos,
                                                 const float4 q, int kneed, float lo, float hi, uint32_t* hw, LST lst,
                                                 int lane, int kListMax, int dbg, const DenseVox& d, int* ns_out,
                                                 int* nc_out, float* L_out, float* U_out) {
  constexpr int kC = stencil_cands<St>();
  uint32_t nib[(kC + 7) / 8];
  uint32_t* const hl = hw + lane;  // this lane's counter column: slot s at hl[64 s]
  StileHist th;
#pragma unroll
  for (int i = 0; i < kStileSlots; ++i) hl[i * 64] = 0u;
  {
    const float sc_ = (float)kStileBins / (hi - lo), off_ = 1.0f - lo * sc_;
    auto body = [&](auto ci, int, float d2) {
      constexpr int c = decltype(ci)::value;
      const int ix = (int)__builtin_amdgcn_fmed3f(fmaf(d2, sc_, off_), 0.0f, (float)(kStileSlots - 1));
      atomicAdd(&hl[ix * 64], 1u);
      if constexpr ((c & 7) == 0)
        nib[c >> 3] = (uint32_t)ix;
      else
        nib[c >> 3] |= (uint32_t)ix << (4 * (c & 7));
      // packed here, not at the list walk (the compiler would keep every
      // candidate's slot live until then)
      asm volatile("" : "+v"(nib[c >> 3]));
    };
    stencil_scan<St>(txy, tz, qs, SY, SZ, xpos, q, body);
  }
#pragma unroll
  for (int i = 0; i < kStileSlots; ++i) th.h[i] = hl[i * 64];
  int total = th.count(-1);
#pragma unroll
  for (int i = 0; i < kStileBins; ++i) total += th.count(i);
  // the k-th beyond R (or below the histogram's range): handed on
  if (total < kneed || th.count(-1) >= kneed) {
    if (d.stats) atomicAdd(&d.stats[7], 1ull);
    return false;
  }
  float L, U;
  int cum, cb, b0;
  if (!hist_locate<StileHist, kStileBins>(th, kneed, th.count(-1), lo, hi, &L, &U, &cum, &cb, &b0)) return false;
  uint32_t h0[kStileSlots];
#pragma unroll
  for (int i = 0; i < kStileSlots; ++i) h0[i] = th.h[i];
  // refinement (a bin holding more than kRefineAt points): rescans re-bin [L, U)
  for (int lvl = 1; cb > kRefineAt && lvl <= kMaxRefine && U > L; ++lvl) {
    lo = L;
    hi = U;
#pragma unroll
    for (int i = 0; i < kStileSlots; ++i) hl[i * 64] = 0u;
    const float sc_ = (float)kStileBins / (hi - lo), off_ = 1.0f - lo * sc_;
    auto body = [&](auto, int, float d2) {
      const int ix = (int)__builtin_amdgcn_fmed3f(fmaf(d2, sc_, off_), 0.0f, (float)(kStileSlots - 1));
      atomicAdd(&hl[ix * 64], 1u);
    };
    stencil_scan<St>(txy, tz, qs, SY, SZ, xpos, q, body);
#pragma unroll
    for (int i = 0; i < kStileSlots; ++i) th.h[i] = hl[i * 64];
    const int below = th.count(-1);
    if (!hist_locate<StileHist, kStileBins>(th, kneed, below, lo, hi, &L, &U, &cum, &cb)) return false;
  }
  *L_out = L;
  *U_out = U * (1.0f - 1.52587890625e-05f);  // U (1 - 2^-16)
  if (dbg == 2) return true;
  // the list: level-0 slots <= b0 + 1 (b0 0-based; slot = bin + 1), as many
  // as the level-0 counts say, in two parts: slots < b0 (bins at least two
  // below the k-th: certain members) in rows [0, ns), slots b0 and b0 + 1 in
  // rows [ns, ns + nc).  The histogram's LDS is free again (its counts are in
  // h0).
  const uint32_t lim = (uint32_t)b0 + 1u, sure = (uint32_t)b0;
  int ns = 0, nc = 0;
#pragma unroll
  for (int i = 0; i < kStileSlots; ++i) {
    ns += (uint32_t)i < sure ? (int)h0[i] : 0;
    nc += (uint32_t)i >= sure && (uint32_t)i <= lim ? (int)h0[i] : 0;
  }
  *ns_out = ns;
  *nc_out = nc;
  if (ns + nc > kListMax) return true;  // the caller hands the query on
  uint16_t* ws = &lst[0][lane];
  uint16_t* wc = &lst[ns][lane];
  auto conv = [&](auto ci, int slot) {
    constexpr int c = decltype(ci)::value;
    const uint32_t v = (nib[c >> 3] >> (4 * (c & 7))) & 15u;
    if (v <= lim) {
      const bool s_ = v < sure;
      *(s_ ? ws : wc) = (uint16_t)slot;
      ws += s_ ? 64 : 0;
      wc += s_ ? 0 : 64;
    }
  };
  asm volatile("" : "+v"(qs), "+v"(SY), "+v"(SZ));
  walk_rows<St, 0>(qs, SY, SZ, xpos, conv);
  return true;
}

// Block coordinates of a stile launch.  part 0: every block of the block box;
// 1: its shell (the blocks on a face of the box: the z end planes, then the
// ring of every plane between); 2: the interior (needs nbx, nby, nbz >= 3).
// The shell holds the table's faces, where the stencil ball is cut and the
// hand-offs arise: launched apart, its hand-off tail runs while the interior
// blocks still stream (normals_dense_vox).
__device__ __forceinline__ void stile_block(const DenseVox& d, int part, int& bx, int& by, int& bz) {
  const int nbx = d.nbx, nby = d.nby, nbz = d.nbz;
  if (part == 0) {
    const int b = xcd_block(blockIdx.x, nbx * nby * nbz);
    bx = b % nbx;
    by = (b / nbx) % nby;
    bz = b / (nbx * nby);
    return;
  }
  const int ix = nbx - 2, iy = nby - 2, iz = nbz - 2;
  if (part == 2) {
    const int t = xcd_block(blockIdx.x, ix * iy * iz);
    bx = 1 + t % ix;
    by = 1 + (t / ix) % iy;
    bz = 1 + t / (ix * iy);
    return;
  }
  const int plane = nbx * nby, ring = plane - ix * iy;
  int t = xcd_block(blockIdx.x, 2 * plane + iz * ring);
  if (t < 2 * plane) {
    bz = t < plane ? 0 : nbz - 1;
    const int r = t % plane;
    bx = r % nbx;
    by = r / nbx;
    return;
  }
  t -= 2 * plane;
  bz = 1 + t / ring;
  int r = t % ring;
  if (r < 2 * nbx) {
    by = r < nbx ? 0 : nby - 1;
    bx = r % nbx;
  } else {
    r -= 2 * nbx;
    by = 1 + (r >> 1);
    bx = (r & 1) ? nbx - 1 : 0;
  }
}

// WPE: waves per SIMD to register-allocate for (LDS allows 3 for 2x2)
template <int KMAX, int WY, int WZ, int WPE>
__global__ void __launch_bounds__(64 * WY * WZ) __attribute__((amdgpu_waves_per_eu(WPE)))
k_normals_stile(DenseVox d, int kneed, const float* __restrict__ prior, float* __restrict__ out,
                int32_t* __restrict__ fb_list, int32_t* __restrict__ fb_len, int force_fb, int dbg, int part) {
  using Sh = StileShape<WY, WZ>;
  constexpr int kSY = Sh::SY, kSZ = Sh::SZ, kSlots = Sh::CELLS;
  __shared__ float2 txy[kSlots];
  __shared__ float tz[kSlots];
  // list capacity: the k - 1 points below the k-th bin + that bin and the next
  // (<= kRefineAt each after refinement) + the rounding band
  constexpr int kListMax = KMAX + kBndCap;
  constexpr int kListWords = ((kListMax + 1) * 64 * (int)sizeof(uint16_t) + 3) / 4;
  constexpr int kHistWords = kStileSlots * 64;
  constexpr int kSelWords = kListWords > kHistWords ? kListWords : kHistWords;
  __shared__ uint32_t selbuf[Sh::NW][kSelWords];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint16_t(*lst)[64] = reinterpret_cast<uint16_t(*)[64]>(selbuf[wv]);
  uint32_t* hw = selbuf[wv];
  int bx, by, bz;
  stile_block(d, part, bx, by, bz);
  const int gx0 = bx * kVB - kVM, gy0 = by * (kVB * WY) - kVM, gz0 = bz * (kVB * WZ) - kVM;  // box origin
  {
    constexpr int kT = 64 * Sh::NW;
    constexpr int J = (Sh::NC + kT - 1) / kT;
    float4 buf[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int t = threadIdx.x + kT * j;
      if (t < Sh::NC) buf[j] = dvox_load(d, gx0 + t % kVE, gy0 + (t / kVE) % Sh::EY, gz0 + t / (kVE * Sh::EY));
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int t = threadIdx.x + kT * j;
      if (t < Sh::NC) {
        const int u = t % (kVE * Sh::EY) + kSZ * (t / (kVE * Sh::EY));  // padded slot
        txy[u] = make_float2(buf[j].x, buf[j].y);
        tz[u] = buf[j].z;
      }
    }
  }
  __syncthreads();
  const int lx = lane & 3, ly = ((lane >> 2) & 3) + kVB * (wv % WY), lz = (lane >> 4) + kVB * (wv / WY);
  const int qs = (lx + kVM) + kSY * (ly + kVM) + kSZ * (lz + kVM);
  const float4 q = make_float4(txy[qs].x, txy[qs].y, tz[qs], 0.0f);
  if (!(q.x < INFINITY)) return;  // empty voxel or outside the grid: no query (no barrier follows)
  const int vx = gx0 + kVM + lx, vy = gy0 + kVM + ly, vz = gz0 + kVM + lz;
  const int64_t vq = vx + (int64_t)d.nx * (vy + (int64_t)d.ny * vz);
  const int oi = __float_as_int(d.vox[vq].w);
  // orientation: the half of its voxel the query lies in, per axis
  const bool xpos = (q.x - (d.ox + (float)vx * d.vs)) * d.inv_vs >= 0.5f;
  const bool ypos = (q.y - (d.oy + (float)vy * d.vs)) * d.inv_vs >= 0.5f;
  const bool zpos = (q.z - (d.oz + (float)vz * d.vs)) * d.inv_vs >= 0.5f;
  const int SY = ypos ? kSY : -kSY, SZ = zpos ? kSZ : -kSZ;
  bool fb = force_fb != 0;  // force_fb: tests of the hand-off path
  if (dbg == 1) {             // profiling only (O3DX_TILE_DEBUG): stop after staging
    if (q.x == 12345.f) out[0] = 0.f;
    return;
  }
  // waves within kEdge voxels of a table face (the cloud's borders of a
  // volumetric cloud) scan the wider 2.45-voxel stencil: there the 2.2 ball is
  // cut by the border and would hand many queries on; a wave-uniform choice
  const int wx0 = gx0 + kVM, wy0 = gy0 + kVM + kVB * (wv % WY), wz0 = gz0 + kVM + kVB * (wv / WY);
  const bool wide = wx0 < kEdge || wy0 < kEdge || wz0 < kEdge || wx0 + kVB > d.nx - kEdge ||
                    wy0 + kVB > d.ny - kEdge || wz0 + kVB > d.nz - kEdge;
  float L = 0.f, U = 0.f;
  int ns = 0, nc = 0;
  if (!fb) {
    if (wide)
      fb = !stile_count_list<Stencil245>(txy, tz, qs, SY, SZ, xpos, q, kneed, d.hlo2, d.rw2, hw, lst, lane, kListMax,
                                         dbg, d, &ns, &nc, &L, &U);
    else
      fb = !stile_count_list<Stencil220>(txy, tz, qs, SY, SZ, xpos, q, kneed, d.hlo2, d.rc2, hw, lst, lane, kListMax,
                                         dbg, d, &ns, &nc, &L, &U);
  }
  if (dbg == 2 || dbg == 3) {
    if (ns + nc == 12345 || L == 12345.f) out[0] = 0.f;  // profiling only: keep the scans alive
    return;
  }
  if (!fb) {
    const bool over = ns + nc > kListMax;
    if (over && d.stats) atomicAdd(&d.stats[5], 1ull);
    fb = over ||
         !stile_finish<KMAX>(
             q, kneed, ns, nc, L, U, lst, lane,
             [&](int p) { return make_float4(txy[p].x, txy[p].y, tz[p], 0.f); }, prior, oi, out, d.nbr,
             [&](int p) {
               const int bz_ = p / kSZ, r = p - bz_ * kSZ, by_ = r / kSY, bx_ = r - by_ * kSY;
               return __float_as_int(
                   d.vox[(gx0 + bx_) + (int64_t)d.nx * ((gy0 + by_) + (int64_t)d.ny * (gz0 + bz_))].w);
             },
             d.kd2, dbg == 4);
  }
  if (fb) {
    if (d.stats) atomicAdd(&d.stats[4], 1ull);
    const int at = atomicAdd(fb_len, 1);
    fb_list[at] = (int32_t)vq;
  }
}

// ---------------------------------------------------------------------------
// KNN normals, wave-per-query form (second level: the queries the tiles hand
// on, or every query when tiles are off).  One wave scans one query's cube
// rows — contiguous ranges of the cell-sorted array, so lanes read coalesced
// — growing S until >= k points lie inside R; per-lane packed 16-bit bin
// counters are summed across the wave; the certain / band lists are built
// with ballot + mbcnt into LDS; the exact tail ranks the band (<= 64, one per
// lane) by (d2_f64, original index); the moments are float64 wave sums.
constexpr int kWaveBnd = 64;
constexpr int kWaveRefineAt = 32;
constexpr int kWavesPerBlock = 4;
constexpr int kWaveCache = 512;  // candidates per wave kept in LDS (d2 + position)

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lanes_below(uint64_t mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Rows of the (2S+1)^3 cube (S <= 5: two rows per lane) into the wave's LDS
// row table: ra = first cell-sorted position, rp = prefix of the row lengths;
// each row is trimmed to the x-cells whose boxes (widened by 2 slack) come
// closer to q than sqrt(r2), rows that do not are dropped.  Returns the
// candidate count.  One round of loads, then every scan walks the rows'
// points as one flat range.
constexpr int kWaveMaxS = 5;
constexpr int kWaveRows = 128;  // >= (2 kWaveMaxS + 1)^2

__device__ __forceinline__ int wave_rows(const GridView& g, const float4 q, int cx, int cy, int cz, int S, float r2,
                                         int lane, int32_t* __restrict__ ra, int32_t* __restrict__ rp) {
  const int side = 2 * S + 1, nr = side * side;
  int carry = 0;
  if (lane == 0) rp[0] = 0;
  for (int h = 0; h * 64 < nr; ++h) {
    const int row = lane + 64 * h;
    int a = 0, len = 0;
    if (row < nr) {
      const int z = cz + row / side - S, y = cy + row % side - S;
      if (z >= 0 && z < g.nz && y >= 0 && y < g.ny) {
        const float y0 = g.oy + (float)y * g.h, z0 = g.oz + (float)z * g.h, sl = 2.0f * g.slack;
        const float dy = fmaxf(fmaxf(y0 - q.y, q.y - (y0 + g.h)) - sl, 0.0f);
        const float dz = fmaxf(fmaxf(z0 - q.z, q.z - (z0 + g.h)) - sl, 0.0f);
        const float rem = r2 - fmaf(dy, dy, dz * dz);
        if (rem > 0.0f) {
          const float rx = sqrtf(rem) + sl;
          const int x0 = max(max(cx - S, 0), (int)floorf((q.x - rx - g.ox) * g.inv_h));
          const int x1 = min(min(cx + S, g.nx - 1), (int)floorf((q.x + rx - g.ox) * g.inv_h));
          if (x0 <= x1) {
            const int rb = g.nx * (y + g.ny * z);
            a = cell_start(g, rb + x0);
            len = cell_start(g, rb + x1 + 1) - a;
          }
        }
      }
    }
    const int inc = wave_incl_scan(len) + carry;
    if (row < nr) {
      ra[row] = a;
      rp[row + 1] = inc;
    }
    carry = __shfl(inc, 63, 64);
  }
  wave_sync();
  return carry;
}

// The cube's candidates as one flat range, 256 per step (four independent
// loads in flight per lane); each lane's row cursor only moves forward.
// `valid` marks lanes past the end; `pp` is the candidate's position.
#define O3DX_WAVE_SCAN(S, BODY)                                                  \
  {                                                                              \
    int row_ = 0;                                                                \
    for (int b_ = 0; b_ < ncand; b_ += 64 * WU) {                                \
      float4 v_[WU];                                                             \
      int p_[WU];                                                                \
      _Pragma("unroll") for (int u_ = 0; u_ < WU; ++u_) {                        \
        const int f_ = b_ + u_ * 64 + lane;                                      \
        p_[u_] = -1;                                                             \
        if (f_ < ncand) {                                                        \
          while (rp[row_ + 1] <= f_) ++row_;                                     \
          p_[u_] = ra[row_] + (f_ - rp[row_]);                                   \
        }                                                                        \
        v_[u_] = g.pts[p_[u_] >= 0 ? p_[u_] : 0];                                \
      }                                                                          \
      _Pragma("unroll") for (int u_ = 0; u_ < WU; ++u_) {                        \
        const int pp = p_[u_];                                                   \
        const bool valid = pp >= 0;                                              \
        const int fidx = b_ + u_ * 64 + lane;                                    \
        const float d2 = dist2_f32(q, v_[u_].x, v_[u_].y, v_[u_].z);             \
        (void)fidx;                                                              \
        BODY                                                                     \
      }                                                                          \
    }                                                                            \
  }

// The same candidates from the wave's LDS cache (filled by the first scan of
// the shell when they fit): no global loads in the refinement / list scans.
#define O3DX_WAVE_SCAN_L(BODY)                                                   \
  for (int b_ = 0; b_ < ncand; b_ += 64) {                                       \
    const int f_ = b_ + lane;                                                    \
    const bool valid = f_ < ncand;                                               \
    const float d2 = valid ? cd2[f_] : 0.0f;                                     \
    const int pp = valid ? cpos[f_] : -1;                                        \
    (void)pp;                                                                    \
    BODY                                                                         \
  }
#define O3DX_WAVE_ANY(BODY)        \
  if (cached) {                    \
    O3DX_WAVE_SCAN_L(BODY)         \
  } else {                         \
    O3DX_WAVE_SCAN(S, BODY)        \
  }

// Moments of the wave form's settled queries, finished lane-parallel by
// k_finish_deferred instead of by lane 0 of each query's wave (FastEigen3x3 in
// float64 is a few hundred serial instructions per query): list slots below
// cap; row -1 = handed on.  cap 0: finish in place.
struct Deferred {
  double* mom = nullptr;  // [9][cap]
  int32_t* row = nullptr;
  int64_t cap = 0;
};

__global__ void __launch_bounds__(kBlock) k_finish_deferred(Deferred df, const int32_t* __restrict__ len, int kneed,
                                                            const float* __restrict__ prior, float* __restrict__ out) {
  const int64_t m = min((int64_t)*len, df.cap);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
    const int row = df.row[t];
    if (row < 0) continue;
    MomAcc acc;
#pragma unroll
    for (int j = 0; j < 9; ++j) acc.m[j] = df.mom[j * df.cap + t];
    finish_normal(kneed, acc, prior, row, out);
  }
}

template <int KMAX, int WU>
__device__ __forceinline__ void wave_query(const GridView& g, int kneed, const float* __restrict__ prior,
                                           float* __restrict__ out, int64_t s, int lane, int32_t* sel, int32_t* bnd,
                                           int32_t* __restrict__ ra, int32_t* __restrict__ rp,
                                           float* __restrict__ cd2, int32_t* __restrict__ cpos,
                                           int32_t* __restrict__ fb_list, int32_t* __restrict__ fb_len, int s0,
                                           const Deferred& df, int64_t t) {
  const float4 q = g.pts[s];
  int cx, cy, cz;
  grid_cell(g, q.x, q.y, q.z, cx, cy, cz);
  const int rmax = shell_rmax(g, cx, cy, cz);
  bool fb = false;
  int S = s0;
  float R2 = 0.f;
  RegHist<false> hist;
  int ncand = 0;
  bool cached = false;
  // A query the tile handed on (s0 = 2) rarely needs more than the shell-1
  // reach + h/2: that ball first (fewer rows and x-cells of the 5^3 cube),
  // then the whole shell.
  // (The stile's hand-offs, s0 = 3, are queries whose k-th neighbour lies
  // beyond its 2.45-voxel stencil — mostly the cube's edges and corners: no
  // trial ball, the shell itself.)
  bool trial = s0 == 2;
  // A dense own cell (a thin plane or a cluster far above the grid's mean
  // occupancy) holds the k nearest within a much smaller ball: a first try at
  // the radius its density suggests (2-D estimate, x2 margin; any radius below
  // the scanned reach is exact, too few points inside just moves on to the
  // shell's own ball).
  float Rd = INFINITY;
  {
    const int c = cell_index(g, cx, cy, cz);
    const int cown = cell_start(g, c + 1) - cell_start(g, c);
    if (cown >= 4 * kneed) Rd = g.h * sqrtf(2.0f * (float)kneed / (float)cown);
  }
  bool dtry = Rd < INFINITY;
  for (;;) {
    if (S >= rmax || S > kWaveMaxS) {  // beyond the row table, or the whole grid: the exact path
      fb = true;
      break;
    }
    double R = cube_reach(g, q.x, q.y, q.z, cx, cy, cz, S) - g.slack;
    if (trial) R = fmin(R, cube_reach(g, q.x, q.y, q.z, cx, cy, cz, S - 1) - g.slack + 0.5 * (double)g.h);
    if (dtry) R = fmin(R, (double)Rd);
    if (R <= 0.0) {
      ++S;
      trial = false;
      dtry = false;
      continue;
    }
    R2 = (float)(R * R) * (1.0f - 4.0f * kRelEps);
    wave_sync();  // the previous shell's row table is no longer read
    ncand = wave_rows(g, q, cx, cy, cz, S, R2, lane, ra, rp);
    cached = ncand <= kWaveCache;
    const float scale = (float)kHistBins / R2;
    hist.zero();
    int tot = 0;
    O3DX_WAVE_SCAN(S, {
      if (cached && valid) {
        cd2[fidx] = d2;
        cpos[fidx] = pp;
      }
      if (valid && d2 < R2) {
        hist.add(min((int)(d2 * scale), kHistBins - 1));
        ++tot;
      }
    })
    tot = wave_sum(tot);
    if (tot > hist.kMaxTotal) {  // packed wave sums could carry
      fb = true;
      break;
    }
    if (tot >= kneed) break;
    if (dtry)
      dtry = false;
    else if (trial)
      trial = false;
    else
      ++S;
  }
  wave_sync();  // the LDS cache is read by other lanes from here on
  float lo = 0.f, hi = R2, L = 0.f, U = 0.f;
  int below = 0;
  for (int lvl = 0; !fb; ++lvl) {
#pragma unroll
    for (int i = 0; i < hist.kWords; ++i) hist.h[i] = wave_sum(hist.h[i]);
    int cum, cb;
    if (!hist_locate(hist, kneed, below, lo, hi, &L, &U, &cum, &cb)) {
      fb = true;
      break;
    }
    if (cb <= kWaveRefineAt || lvl == kMaxRefine || !(U > L)) break;
    below += cum;
    lo = L;
    hi = U;
    const float sc = (float)kHistBins / (hi - lo);
    hist.zero();
    O3DX_WAVE_ANY(if (valid && d2 >= lo && d2 < hi) hist.add(min((int)((d2 - lo) * sc), kHistBins - 1));)
  }
  int nsel = 0, nb = 0;
  if (!fb) {
    const float Lm = L * (1.0f - 2.0f * kRelEps), Up = U * (1.0f + 2.0f * kRelEps);
    int nU = 0;
    O3DX_WAVE_ANY({
      nU += __popcll(__ballot(valid && d2 < U));
      const bool c1 = valid && d2 < Lm;
      const bool c2 = valid && !(d2 < Lm) && d2 < Up;
      const uint64_t m1 = __ballot(c1);
      const uint64_t m2 = __ballot(c2);
      if (c1) {
        const int at = nsel + lanes_below(m1);
        if (at < KMAX) sel[at] = pp;
      }
      if (c2) {
        const int at = nb + lanes_below(m2);
        if (at < kWaveBnd) bnd[at] = pp;
      }
      nsel += __popcll(m1);
      nb += __popcll(m2);
    })
    fb = nsel > kneed || nb > kWaveBnd || nsel + nb < kneed || nU < kneed;
  }
  if (!fb) {
    wave_sync();
    const int need = kneed - nsel;
    const double qx = q.x, qy = q.y, qz = q.z;
    // exact keys of the band, one per lane, and their ranks
    double bd = INFINITY;
    int bid = 0x7fffffff, bpos = -1;
    if (lane < nb) {
      bpos = bnd[lane];
      const float4 v = g.pts[bpos];
      bd = dist2_f64(qx, qy, qz, v);
      bid = __float_as_int(v.w);
    }
    int rank = 0;
    for (int i = 0; i < nb; ++i) {
      const double di = __shfl(bd, i, 64);
      const int ii = __shfl(bid, i, 64);
      rank += (di < bd || (di == bd && ii < bid)) ? 1 : 0;
    }
    // largest certain key must precede the smallest unselected band key (rank == need)
    double cd = -1.0;
    int cid = -1;
    if (lane < nsel) {
      const float4 v = g.pts[sel[lane]];
      cd = dist2_f64(qx, qy, qz, v);
      cid = __float_as_int(v.w);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double od = __shfl_xor(cd, o, 64);
      const int oid = __shfl_xor(cid, o, 64);
      if (od > cd || (od == cd && oid > cid)) {
        cd = od;
        cid = oid;
      }
    }
    if (need < nb && nsel > 0) {
      const uint64_t mk = __ballot(lane < nb && rank == need);
      const int l = __ffsll((unsigned long long)mk) - 1;
      const double ud = __shfl(bd, l, 64);
      const int uid = __shfl(bid, l, 64);
      fb = !(cd < ud || (cd == ud && cid < uid));
    }
    if (!fb) {
      if (lane < nb && rank < need) sel[nsel + rank] = bpos;
      wave_sync();
      double x = 0.0, y = 0.0, z = 0.0;
      if (lane < kneed) {
        const float4 v = g.pts[sel[lane]];
        x = v.x;
        y = v.y;
        z = v.z;
        if (g.nbr) g.nbr[(int64_t)__float_as_int(q.w) * kneed + lane] = __float_as_int(v.w);
      }
      if (g.kd2) {
        double dk = lane < kneed ? dist2_f64(q.x, q.y, q.z, g.pts[sel[lane]]) : 0.0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) dk = fmax(dk, __shfl_xor(dk, o, 64));
        if (lane == 0) g.kd2[__float_as_int(q.w)] = (float)(dk * (1.0 + 1e-6));
      }
      // exact sums over the lanes (MomAccDD): the lane a neighbour landed on
      // (the scan order) does not change the bits
      MomAcc acc;
      const double t9[9] = {x, y, z, x * x, x * y, x * z, y * y, y * z, z * z};
#pragma unroll
      for (int j = 0; j < 9; ++j) acc.m[j] = wave_sum_exact(t9[j]);
      if (lane == 0) {
        if (t < df.cap) {  // the eigen solve runs lane-parallel afterwards (k_finish_deferred)
#pragma unroll
          for (int j = 0; j < 9; ++j) df.mom[j * df.cap + t] = acc.m[j];
          df.row[t] = __float_as_int(q.w);
        } else {
          finish_normal(kneed, acc, prior, __float_as_int(q.w), out);
        }
      }
    }
  }
  wave_sync();  // the lists are reused by the wave's next query
  if (fb && lane == 0) {
    if (t < df.cap) df.row[t] = -1;
    if (g.stats) atomicAdd(&g.stats[5], 1ull);
    const int at = atomicAdd(fb_len, 1);
    fb_list[at] = (int32_t)s;
  }
}
#undef O3DX_WAVE_SCAN
#undef O3DX_WAVE_SCAN_L
#undef O3DX_WAVE_ANY

template <int KMAX, int WU = 4>
__global__ void __launch_bounds__(64 * kWavesPerBlock) __attribute__((amdgpu_waves_per_eu(4))) k_normals_knn_wave(
    GridView g, int kneed, const float* __restrict__ prior, float* __restrict__ out,
    const int32_t* __restrict__ in_list, const int32_t* __restrict__ in_len, int32_t* __restrict__ fb_list,
    int32_t* __restrict__ fb_len, int s0, Deferred df) {
  __shared__ int32_t sel[kWavesPerBlock][KMAX];
  __shared__ int32_t bnd[kWavesPerBlock][kWaveBnd];
  __shared__ int32_t ra[kWavesPerBlock][kWaveRows];
  __shared__ int32_t rp[kWavesPerBlock][kWaveRows + 1];
  __shared__ float cd2[kWavesPerBlock][kWaveCache];
  __shared__ int32_t cpos[kWavesPerBlock][kWaveCache];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t lim = in_list ? (int64_t)*in_len : g.n;
  for (int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + wv; t < lim; t += (int64_t)gridDim.x * kWavesPerBlock) {
    const int64_t s = in_list ? (int64_t)__builtin_amdgcn_readfirstlane(in_list[t]) : t;
    wave_query<KMAX, WU>(g, kneed, prior, out, s, lane, sel[wv], bnd[wv], ra[wv], rp[wv], cd2[wv], cpos[wv], fb_list,
                         fb_len, s0, df, t);
  }
}

__global__ void __launch_bounds__(kBlock) k_normals_radius(GridView g, double radius, const float* __restrict__ prior,
                                                           float* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.n) return;
  const float4 q = g.pts[s];
  const int oi = __float_as_int(q.w);
  int cx, cy, cz;
  grid_cell(g, q.x, q.y, q.z, cx, cy, cz);
  const int rmax = shell_rmax(g, cx, cy, cz);
  const double r2 = radius * radius, qx = q.x, qy = q.y, qz = q.z;
  MomAccDD acc;
  acc.zero();
  int cnt = 0;
  for (int r = 0; r <= rmax; ++r) {
    for_shell(g, cx, cy, cz, r, [&](int c) {
      const int s1 = g.start[c + 1];
      for (int p = g.start[c]; p < s1; ++p) {
        const float4 v = g.pts[p];
        if (dist2_f64(qx, qy, qz, v) < r2) {
          acc.add((double)v.x, (double)v.y, (double)v.z);
          ++cnt;
        }
      }
    });
    if (cube_reach(g, qx, qy, qz, cx, cy, cz, r) - g.slack >= radius) break;
  }
  finish_normal(cnt, acc, prior, oi, out);
}

template <int K>
__global__ void __launch_bounds__(kBlock) k_knn_query(GridView g, const float* __restrict__ q, int64_t nq, int kneed,
                                                      int hybrid, double radius, int kout,
                                                      int32_t* __restrict__ idx_out, double* __restrict__ d2_out,
                                                      int32_t* __restrict__ cnt_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  double bd[K];
  int bi[K];
  const int cnt = knn_search_dev<K>(g, q[3 * i], q[3 * i + 1], q[3 * i + 2], kneed, hybrid != 0, radius, bd, bi);
  cnt_out[i] = cnt;
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (j < kout) {
      idx_out[i * kout + j] = j < cnt ? bi[j] : -1;
      if (d2_out) d2_out[i * kout + j] = j < cnt ? bd[j] : INFINITY;
    }
}

static int pick_k(int k) {
  if (k <= 4) return 4;
  if (k <= 8) return 8;
  if (k <= 16) return 16;
  if (k <= 32) return 32;
  return 64;
}

#define O3DX_DISPATCH_K(kk, KERNEL, ...)                                                          \
  switch (pick_k(kk)) {                                                                           \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                                   \
    case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                                   \
    case 16: hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__); break;                                 \
    case 32: hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__); break;                                 \
    default: hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__); break;                                 \
  }

// grid occupancy target per search mode: ~k/4 points per cell keeps the
// 27-cell first shell close to 2-3 k candidates
static double occ_for(int mode, int k) {
  if (mode == O3DX_SEARCH_RADIUS) return 4.0;
  if (mode == O3DX_SEARCH_KNN) return std::max(4.0, k / 3.0);  // histogram path: shells 0..1 hold k
  return std::max(2.0, k / 4.0);
}

// ------------------------------------------------------ grid from voxels
// Search grid read off a voxel table (o3dx_voxel_down_sample_grid): cell =
// b^3 voxels, origin = the voxel grid's min_bound, each cell's points in voxel
// order (x fastest) — a count and an emit pass over the table, no sort.  The
// cell of a point is fixed by its float64 voxel key; the float32 cell test of
// the search kernels sees the same faces up to rounding, covered by `slack`
// exactly as for grid_build's own float32 assignment.
template <int B>
__global__ void __launch_bounds__(kBlock) k_vgrid_count(const float4* __restrict__ vox, int vnx, int vny, int vnz,
                                                        GridView g, int32_t* __restrict__ count) {
  const int64_t nc = (int64_t)g.nx * g.ny * g.nz;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x) {
    const int cx = (int)(c % g.nx), cy = (int)((c / g.nx) % g.ny), cz = (int)(c / ((int64_t)g.nx * g.ny));
    int k = 0;
    for (int dz = 0; dz < B; ++dz)
      for (int dy = 0; dy < B; ++dy)
#pragma unroll
        for (int dx = 0; dx < B; ++dx) {
          const int x = cx * B + dx, y = cy * B + dy, z = cz * B + dz;
          if (x < vnx && y < vny && z < vnz)
            k += __float_as_int(vox[x + (int64_t)vnx * (y + (int64_t)vny * z)].w) >= 0;
        }
    count[c] = k;
  }
}

template <int B>
__global__ void __launch_bounds__(kBlock) k_vgrid_emit(const float4* __restrict__ vox, int vnx, int vny, int vnz,
                                                       GridView g, float4* __restrict__ pts) {
  const int64_t nc = (int64_t)g.nx * g.ny * g.nz;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x) {
    const int cx = (int)(c % g.nx), cy = (int)((c / g.nx) % g.ny), cz = (int)(c / ((int64_t)g.nx * g.ny));
    int p = g.start[c];
    for (int dz = 0; dz < B; ++dz)
      for (int dy = 0; dy < B; ++dy)
#pragma unroll
        for (int dx = 0; dx < B; ++dx) {
          const int x = cx * B + dx, y = cy * B + dy, z = cz * B + dz;
          if (x >= vnx || y >= vny || z >= vnz) continue;
          const float4 v = vox[x + (int64_t)vnx * (y + (int64_t)vny * z)];
          if (__float_as_int(v.w) >= 0) pts[p++] = v;
        }
  }
}

// 0: built; 1: no usable voxel grid (caller sorts the points instead).
static int grid_from_voxels(const double* geom, const float4* vox, int64_t n, double target_occ, void* ws,
                            size_t ws_bytes, hipStream_t s, GridBuild* out) {
  if (!vox || geom[7] != 1.0) return 1;
  const int vn[3] = {(int)geom[4], (int)geom[5], (int)geom[6]};
  const double vs = geom[3];
  GridLayout L = grid_layout(n, 4);
  if (ws_bytes < L.total) return fail(O3DX_ENOMEM, "grid workspace too small (need %zu)", L.total);
  // b: mean points per occupied cell closest to the target.  One rep per
  // occupied voxel and the occupied 2^3 cells give the cloud's local
  // dimension D = log2(m / occ2); a cell of b^3 voxels then holds ~b^D reps.
  const double occ2 = geom[8];
  if (!(occ2 > 0.0)) return 1;
  const double D = std::min(3.0, std::max(1.0, std::log2((double)n / occ2)));
  int b = 0;
  double best = 0.0;
  for (int c = 1; c <= 4; ++c) {
    int64_t cells = 1;
    for (int a = 0; a < 3; ++a) cells *= (vn[a] + c - 1) / c;
    if (cells > cap_cells(n, 4)) continue;
    const double err = std::fabs(D * std::log((double)c) - std::log(target_occ));
    if (b == 0 || err < best) {
      b = c;
      best = err;
    }
  }
  if (b == 0) return 1;
  char* w = (char*)ws;
  GridBuild& G = *out;
  G.pts = (float4*)(w + L.pts);
  G.start = (int32_t*)(w + L.start);
  G.count = (int32_t*)(w + L.count);
  G.cell = (int32_t*)(w + L.cell);
  G.rank = (int32_t*)(w + L.rank);
  G.scan_tmp = (int32_t*)(w + L.scan);
  G.aabb_ws = w + L.aabb;
  G.mm = (double*)(w + L.mm);
  G.scratch = (int64_t*)(w + L.scratch);
  G.cap_cells = cap_cells(n, 4);
  G.extra = nullptr;
  GridView& g = G.view;
  const double h = b * vs;
  double maxabs = 0.0, maxext = 0.0;
  for (int a = 0; a < 3; ++a) {
    const double ext = vn[a] * vs;
    maxabs = std::max(maxabs, std::max(std::fabs(geom[a]), std::fabs(geom[a] + ext)));
    maxext = std::max(maxext, ext);
  }
  g.pts = G.pts;
  g.start = G.start;
  g.ox = (float)geom[0];
  g.oy = (float)geom[1];
  g.oz = (float)geom[2];
  g.h = (float)h;
  g.inv_h = (float)(1.0 / h);
  g.nx = (vn[0] + b - 1) / b;
  g.ny = (vn[1] + b - 1) / b;
  g.nz = (vn[2] + b - 1) / b;
  g.n = n;
  g.stats = search_stats_ptr();
  g.slack = (float)(32.0 * std::ldexp(1.0, -24) * (maxabs + maxext) + 1e-6 * h);
  g.blocked = 0;
  g.bnx = (g.nx + 7) / 8;
  g.bny = (g.ny + 7) / 8;
  const int64_t nc = (int64_t)g.nx * g.ny * g.nz;
  const unsigned gc = grid_for(nc, kBlock, 8192);
  KTimer kt("grid_voxel", s);
  switch (b) {
#define O3DX_VGRID(BB)                                                                                          \
  case BB:                                                                                                      \
    hipLaunchKernelGGL(k_vgrid_count<BB>, dim3(gc), dim3(kBlock), 0, s, vox, vn[0], vn[1], vn[2], g, G.count);  \
    O3DX_TRY(exclusive_scan_i32(G.count, G.start, nc, G.scan_tmp, s));                                          \
    hipLaunchKernelGGL(k_vgrid_emit<BB>, dim3(gc), dim3(kBlock), 0, s, vox, vn[0], vn[1], vn[2], g, G.pts);      \
    break;
    O3DX_VGRID(1)
    O3DX_VGRID(2)
    O3DX_VGRID(3)
    O3DX_VGRID(4)
#undef O3DX_VGRID
  }
  O3DX_HIP(hipGetLastError());
  return 0;
}

// A second stream per host thread and device (created on first use, kept for
// the thread's life): the stile's shell blocks and their hand-off tail run
// there beside the interior blocks.  nullptr (no split) when `s` is not on
// the current device or creation fails.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, a_done = nullptr, join = nullptr;
};
static SideStream* side_stream(hipStream_t s) {
  constexpr int kMaxDev = 64;
  static thread_local SideStream tab[kMaxDev];
  int cur = -1;
  hipDevice_t sd = -1;
  if (hipGetDevice(&cur) != hipSuccess || hipStreamGetDevice(s, &sd) != hipSuccess || sd != cur || cur < 0 ||
      cur >= kMaxDev)
    return nullptr;
  SideStream& x = tab[cur];
  if (!x.s) {
    SideStream y;
    if (hipStreamCreateWithFlags(&y.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&y.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&y.a_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&y.join, hipEventDisableTiming) != hipSuccess) {
      for (hipEvent_t e : {y.fork, y.a_done, y.join})
        if (e) (void)hipEventDestroy(e);
      (void)hipStreamDestroy(y.s);
      return nullptr;
    }
    x = y;
  }
  return &x;
}

// KNN normals straight off the dense voxel table (k_normals_stile; hand-offs
// to the wave form and the register top-k over the table).  1: not applicable
// (the caller builds a search grid instead).
// Whether the normals run straight off the voxel table: KNN with k <= 32 and
// representatives filling their voxels (occupied fraction of the voxels in
// occupied 2^3 cells >= 0.7, so the stencil ball (2.45 voxels) holds the k
// nearest with a wide margin).  *kth: the expected k-th distance (voxels).
static bool dense_vox_applicable(const double* geom, const float4* vox, int64_t n, int mode, int knn, double* kth) {
  if (!vox || geom[7] != 1.0 || mode != O3DX_SEARCH_KNN || getenv("O3DX_NO_STILE")) return false;
  const int kneed = (int)std::min<int64_t>(knn, n);
  if (kneed < 1 || kneed > 32) return false;
  if (geom[8] == -1.0) {  // o3dx_voxel_table_build_deferred: occupancy not measured
    *kth = std::cbrt((double)kneed / 4.18879020478639098);
    return true;
  }
  if (!(geom[8] > 0.0)) return false;
  const double dens = (double)n / (8.0 * geom[8]);
  *kth = std::cbrt((double)kneed / (std::min(dens, 1.0) * 4.18879020478639098));
  return dens >= 0.7 && *kth <= 2.0;
}

// spec: launched before the voxel counts are read back (o3dx_voxel_down_sample_normals):
// n is then only the capacity (rows < n), kneed = knn, and the caller checks
// dense_vox_applicable once the counts are known.
static int normals_dense_vox(const double* geom, const float4* vox, const float* xyz, int64_t n, int mode, int knn,
                             const float* prior, float* out, float* kd2, void* ws, size_t ws_bytes, hipStream_t s,
                             bool spec = false, bool lens_zeroed = false) {
  double kth = 0.0;
  int kneed = knn;
  if (spec) {
    if (!vox || mode != O3DX_SEARCH_KNN || knn < 1 || knn > 32 || n < knn || getenv("O3DX_NO_STILE")) return 1;
    kth = std::cbrt((double)knn / 4.18879020478639098);
  } else {
    if (!dense_vox_applicable(geom, vox, n, mode, knn, &kth)) return 1;
    kneed = (int)std::min<int64_t>(knn, n);
  }
  DenseVox d;
  d.vox = vox;
  d.nx = (int)geom[4];
  d.ny = (int)geom[5];
  d.nz = (int)geom[6];
  // 2 x 2 waves per workgroup sharing one staged box, registers for 3 waves / SIMD
  constexpr int wy = 2, wz = 2;
  d.nbx = (d.nx + kVB - 1) / kVB;
  d.nby = (d.ny + kVB * wy - 1) / (kVB * wy);
  d.nbz = (d.nz + kVB * wz - 1) / (kVB * wz);
  const int64_t nb = (int64_t)d.nbx * d.nby * d.nbz;
  if (nb <= 0 || nb > INT32_MAX || (int64_t)d.nx * d.ny * d.nz > INT32_MAX) return 1;
  d.ox = (float)geom[0];
  d.oy = (float)geom[1];
  d.oz = (float)geom[2];
  d.vs = (float)geom[3];
  d.inv_vs = (float)(1.0 / geom[3]);
  double maxabs = 0.0, maxext = 0.0;
  const int vn[3] = {d.nx, d.ny, d.nz};
  for (int a = 0; a < 3; ++a) {
    const double ext = vn[a] * geom[3];
    maxabs = std::max(maxabs, std::max(std::fabs(geom[a]), std::fabs(geom[a] + ext)));
    maxext = std::max(maxext, ext);
  }
  const double slack = 32.0 * std::ldexp(1.0, -24) * (maxabs + maxext) + 1e-6 * geom[3];
  // completeness radii of the count (2.2 voxels) and the smaller list stencil
  // (2.1), shrunk by the float32 slack; the histogram's lower edge (1.5 voxels)
  const double R = kStencilR * geom[3] - slack, Rl = kListR * geom[3] - slack;
  d.rc2 = (float)(R * R) * (1.0f - 4.0f * kRelEps);
  d.rl2 = (float)(Rl * Rl) * (1.0f - 4.0f * kRelEps);
  const double Rw = kWideR * geom[3] - slack;
  d.rw2 = (float)(Rw * Rw) * (1.0f - 4.0f * kRelEps);
  d.hlo2 = (float)(kHistLo * geom[3] * kHistLo * geom[3]);
  d.stats = search_stats_ptr();
  d.nbr = debug_nbr(kneed, n);
  d.kd2 = kd2;
  Arena ar((char*)ws, ws_bytes);
  int32_t* lens = ar.take<int32_t>(4);
  int32_t* list = ar.take<int32_t>(n);
  int32_t* list2 = ar.take<int32_t>(n);
  O3DX_ARENA_CHECK(ar);
  // (the one-call pipeline clears them in its bounds pass: no fill launch here)
  if (!lens_zeroed) O3DX_HIP(hipMemsetAsync(lens, 0, 4 * sizeof(int32_t), s));
  // Split launch (opt-in, O3DX_STILE_SPLIT=1; a block box of >= 3 blocks per
  // axis): the shell blocks on a side stream, launched first, then their
  // hand-off tail there, while the interior blocks run on s; the interior's
  // own hand-offs follow on s.  Measured at C2 (profiles/r06_stile_split_ab.txt):
  // 0.776 ms per step against 0.755 in one launch — the two concurrent
  // launches stretched the stile 0.470 -> 0.511 ms, and the interior still
  // hands on a few queries, so a 27 us tail stays on the critical path.
  // The interior's hand-offs go to lists of their own (list3 / list4,
  // counters lens[2] / lens[3]).
  const int64_t nint = (int64_t)std::max(d.nbx - 2, 0) * std::max(d.nby - 2, 0) * std::max(d.nbz - 2, 0);
  SideStream* side = nullptr;
  int32_t *list3 = nullptr, *list4 = nullptr;
  const char* want = getenv("O3DX_STILE_SPLIT");
  if (d.nbx >= 3 && d.nby >= 3 && d.nbz >= 3 && want && want[0] == '1') {
    list3 = ar.take<int32_t>(n);  // the interior's hand-off lists
    list4 = ar.take<int32_t>(n);
    if (ar.ok()) side = side_stream(s);
  }
  {
    KTimer kt("normals_knn", s);
    // O3DX_TILE_DEBUG=1/2/3/4: stop after staging / histogram / list scan / moments (profiling only)
    const char* dbg = getenv("O3DX_TILE_DEBUG");
    const int ffb = getenv("O3DX_STILE_FORCE_FB") ? 1 : 0, dg = dbg ? atoi(dbg) : 0;
    KTimer kt_tile("normals_stile", s);
    if (side) {
      O3DX_HIP(hipEventRecord(side->fork, s));
      O3DX_HIP(hipStreamWaitEvent(side->s, side->fork, 0));
      hipLaunchKernelGGL((k_normals_stile<32, wy, wz, 3>), dim3((unsigned)(nb - nint)), dim3(64 * wy * wz), 0,
                         side->s, d, kneed, prior, out, list, lens, ffb, dg, 1);
      O3DX_HIP(hipEventRecord(side->a_done, side->s));
      hipLaunchKernelGGL((k_normals_stile<32, wy, wz, 3>), dim3((unsigned)nint), dim3(64 * wy * wz), 0, s, d, kneed,
                         prior, out, list3, lens + 2, ffb, dg, 2);
      O3DX_HIP(hipStreamWaitEvent(s, side->a_done, 0));
    } else {
      hipLaunchKernelGGL((k_normals_stile<32, wy, wz, 3>), dim3((unsigned)nb), dim3(64 * wy * wz), 0, s, d, kneed,
                         prior, out, list, lens, ffb, dg, 0);
    }
    kt_tile.stop();
    // the table as a dense GridView (identity cell starts, <= 1 point per cell)
    GridView g{};
    g.pts = vox;
    g.start = nullptr;
    g.dense = 1;
    g.ox = (float)geom[0];
    g.oy = (float)geom[1];
    g.oz = (float)geom[2];
    g.h = (float)geom[3];
    g.inv_h = (float)(1.0 / geom[3]);
    g.slack = (float)slack;
    g.nx = d.nx;
    g.ny = d.ny;
    g.nz = d.nz;
    g.n = (int64_t)d.nx * d.ny * d.nz;
    g.stats = d.stats;
    g.nbr = d.nbr;
    g.kd2 = d.kd2;
    auto tail = [&](hipStream_t st, int32_t* l1, int32_t* n1, int32_t* l2, int32_t* n2) {
      hipLaunchKernelGGL(k_normals_knn_wave<32>, dim3(2048), dim3(64 * kWavesPerBlock), 0, st, g, kneed, prior, out,
                         l1, n1, l2, n2, 3, Deferred{});
      hipLaunchKernelGGL(k_normals_knn<32>, dim3(64), dim3(kBlock), 0, st, g, xyz, kneed, 0, 0.0, prior, out, l2,
                         n2);
    };
    if (side) {
      tail(side->s, list, lens, list2, lens + 1);
      O3DX_HIP(hipEventRecord(side->join, side->s));
      KTimer kt_wave("normals_wave", s);
      tail(s, list3, lens + 2, list4, lens + 3);
      kt_wave.stop();
      O3DX_HIP(hipStreamWaitEvent(s, side->join, 0));
    } else {
      KTimer kt_wave("normals_wave", s);
      tail(s, list, lens, list2, lens + 1);
    }
  }
  O3DX_HIP(hipGetLastError());
  return 0;
}

// The normals on a built grid: shared by o3dx_estimate_normals (grid sorted
// from the points) and o3dx_estimate_normals_voxel (grid read off the voxel
// table).  `xyz` is the caller's point array the grid's w fields index.
// ------------------------------------------------------------ nested grids
// A cloud of mixed density (a thin dense plane or cluster inside a sparse
// volume: raw scans, C3's planted plane) puts hundreds of points in the outer
// grid's cells there: their LDS tiles overflow and every such query would go
// to the one-wave-per-query form, whose candidate count grows with the cell
// size (round 3: 2.65M of C3's 10M queries, 37 of 44 ms).  Those queries are
// served instead by a nested grid: the dense cells (>= t points) and their 26
// neighbours (D1) are its queries, the cells within two of a dense cell (D2)
// its points; same tile kernel, cells sized for the dense region, every
// search capped at the outer shell-1 reach (the 27 cells around a D1 cell lie
// in D2, so every point inside that reach is in the nested grid); what it
// cannot settle goes to the outer wave form.
constexpr int64_t kNestedMinQueries = 4096;

// f(c') over the <= 27 cells around cell c of a row-major grid
template <class F>
__device__ __forceinline__ bool any_around(const GridView& g, int64_t c, F&& f) {
  const int cx = (int)(c % g.nx), cy = (int)((c / g.nx) % g.ny), cz = (int)(c / ((int64_t)g.nx * g.ny));
  for (int z = max(cz - 1, 0); z <= min(cz + 1, g.nz - 1); ++z)
    for (int y = max(cy - 1, 0); y <= min(cy + 1, g.ny - 1); ++y)
      for (int x = max(cx - 1, 0); x <= min(cx + 1, g.nx - 1); ++x)
        if (f((int64_t)x + (int64_t)g.nx * (y + (int64_t)g.ny * z))) return true;
  return false;
}

// points in cells of >= t points (one read per cell: the trigger test)
__global__ void __launch_bounds__(kBlock) k_dense_points(GridView g, int t, unsigned long long* __restrict__ tot) {
  const int64_t nc = (int64_t)g.nx * g.ny * g.nz;
  unsigned long long b = 0;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x) {
    const int own = g.start[c + 1] - g.start[c];
    b += own >= t ? (unsigned long long)own : 0ull;
  }
  b = wave_sum(b);
  if (lane_id() == 0 && b) atomicAdd(tot, b);
}

__global__ void __launch_bounds__(kBlock) k_nested_mark(GridView g, int t, uint8_t* __restrict__ d1) {
  const int64_t nc = (int64_t)g.nx * g.ny * g.nz;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x)
    d1[c] = any_around(g, c, [&](int64_t o) { return g.start[o + 1] - g.start[o] >= t; }) ? 1 : 0;
}

__global__ void __launch_bounds__(kBlock) k_nested_cells(GridView g, const uint8_t* __restrict__ d1,
                                                         int32_t* __restrict__ sub_cnt,
                                                         unsigned long long* __restrict__ tot) {
  const int64_t nc = (int64_t)g.nx * g.ny * g.nz;
  unsigned long long a = 0, b = 0;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x) {
    const int own = g.start[c + 1] - g.start[c];
    const bool d2 = own > 0 && any_around(g, c, [&](int64_t o) { return d1[o] != 0; });
    sub_cnt[c] = d2 ? own : 0;
    a += d2 ? (unsigned long long)own : 0ull;
    b += d1[c] ? (unsigned long long)own : 0ull;
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane_id() == 0 && (a | b)) {
    atomicAdd(&tot[0], a);
    atomicAdd(&tot[1], b);
  }
}

// The nested grid's input: the points of the D2 cells, in outer order, with
// w = outer position (a query: D1) or -(position + 1).
__global__ void __launch_bounds__(kBlock) k_nested_gather(GridView g, const uint8_t* __restrict__ d1,
                                                          const int32_t* __restrict__ sub_cnt,
                                                          const int32_t* __restrict__ sub_off,
                                                          float* __restrict__ sub_xyz, int32_t* __restrict__ sub_id) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < g.n; p += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = g.pts[p];
    int cx, cy, cz;
    grid_cell(g, v.x, v.y, v.z, cx, cy, cz);
    const int c = cell_index(g, cx, cy, cz);
    if (sub_cnt[c] == 0) continue;
    const int64_t d = (int64_t)sub_off[c] + (p - g.start[c]);
    sub_xyz[3 * d] = v.x;
    sub_xyz[3 * d + 1] = v.y;
    sub_xyz[3 * d + 2] = v.z;
    sub_id[d] = d1[c] ? (int32_t)p : -(int32_t)p - 1;
  }
}

struct NestedWs {
  int32_t *sub_cnt, *sub_off, *scan_tmp, *chunks;
  uint8_t* d1;
  unsigned long long* tot;
  float* sub_xyz;
  int32_t* sub_id;
  void *gws, *pws;
  size_t gws_bytes, pws_bytes;
  int64_t cap;  // nested points
};

static void nested_carve(Arena& ar, int64_t n, NestedWs& w) {
  const int64_t nc = cap_cells(std::max<int64_t>(n, 1), 4);
  w.cap = n / 2 + 4096;
  w.d1 = ar.take<uint8_t>(nc + 1);
  w.sub_cnt = ar.take<int32_t>(nc + 1);
  w.sub_off = ar.take<int32_t>(nc + 1);
  w.scan_tmp = ar.take<int32_t>(scan_workspace_ints(nc + 1));
  w.tot = ar.take<unsigned long long>(3);
  w.sub_xyz = ar.take<float>(3 * w.cap);
  w.sub_id = ar.take<int32_t>(w.cap);
  w.gws_bytes = grid_ws_bytes(w.cap);
  w.gws = ar.take<char>(w.gws_bytes);
  const int64_t rows = cap_cells(w.cap, 4);
  w.chunks = ar.take<int32_t>(w.cap / kTileQ + rows + 4);
  w.pws_bytes = chunk_plan_ws_bytes(w.cap, rows);
  w.pws = ar.take<char>(w.pws_bytes);
}

static size_t nested_ws_bytes(int64_t n) {
  Arena ar(nullptr, 0);
  NestedWs w;
  nested_carve(ar, n, w);
  return ar.used;
}

// Builds the nested grid and runs its tiles (hand-offs appended to fb_list as
// outer positions); on return G.view.skip_cells tells the outer tiles which
// queries are taken.  Does nothing when the cloud has no dense cells.
static int nested_tiles(GridBuild& G, int64_t n, int kneed, double occ, const float* prior, float* out,
                        int32_t* fb_list, int32_t* fb_len, Arena& ar, hipStream_t s) {
  NestedWs w;
  nested_carve(ar, n, w);
  O3DX_ARENA_CHECK(ar);
  const int t = (int)std::ceil(4.0 * occ);
  const int64_t nc = (int64_t)G.view.nx * G.view.ny * G.view.nz;
  KTimer kt("normals_nested", s);
  O3DX_HIP(hipMemsetAsync(w.tot, 0, 3 * sizeof(unsigned long long), s));
  const unsigned gc = grid_for(nc, kBlock, 4096);
  // worth a second grid only when the dense cells hold a real share of the
  // queries (a surface's edges and corners, a few denser cells, are cheaper
  // left to the outer tiles and the wave form)
  hipLaunchKernelGGL(k_dense_points, dim3(gc), dim3(kBlock), 0, s, G.view, t, w.tot + 2);
  unsigned long long dense = 0;
  O3DX_TRY(read_back(&dense, w.tot + 2, sizeof(dense), s));
  const int64_t minq = std::max<int64_t>(kNestedMinQueries, n / 32);
  if ((int64_t)dense < minq) return 0;
  hipLaunchKernelGGL(k_nested_mark, dim3(gc), dim3(kBlock), 0, s, G.view, t, w.d1);
  hipLaunchKernelGGL(k_nested_cells, dim3(gc), dim3(kBlock), 0, s, G.view, w.d1, w.sub_cnt, w.tot);
  unsigned long long tot[2];
  O3DX_TRY(read_back(tot, w.tot, sizeof(tot), s));
  const int64_t nsub = (int64_t)tot[0];
  if (nsub > w.cap) return 0;
  O3DX_TRY(exclusive_scan_i32(w.sub_cnt, w.sub_off, nc, w.scan_tmp, s));
  hipLaunchKernelGGL(k_nested_gather, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, G.view, w.d1, w.sub_cnt,
                     w.sub_off, w.sub_xyz, w.sub_id);
  GridBuild N;
  O3DX_TRY(grid_build(w.sub_xyz, nsub, occ, 0.0, w.gws, w.gws_bytes, s, &N, nullptr, nullptr, false, 4, false,
                      w.sub_id, 0.5 * (double)G.view.h));
  GridView& v = N.view;
  v.outer = G.view.pts;
  v.cox = G.view.ox;
  v.coy = G.view.oy;
  v.coz = G.view.oz;
  v.ch = G.view.h;
  v.cinv_h = G.view.inv_h;
  v.cslack = G.view.slack;
  v.cnx = G.view.nx;
  v.cny = G.view.ny;
  v.cnz = G.view.nz;
  v.nbr = G.view.nbr;
  v.kd2 = G.view.kd2;
  O3DX_TRY(chunk_plan(nsub, v, kTileQ, w.chunks, w.pws, w.pws_bytes, s));
  const int64_t upper = chunk_plan_upper(nsub, v, kTileQ);
  if (kneed <= 32)
    hipLaunchKernelGGL(k_normals_knn_tile<32>, dim3((unsigned)upper), dim3(kTileQ), 0, s, v, w.chunks, kneed, prior,
                       out, fb_list, fb_len, 0);
  else
    hipLaunchKernelGGL(k_normals_knn_tile<64>, dim3((unsigned)upper), dim3(kTileQ), 0, s, v, w.chunks, kneed, prior,
                       out, fb_list, fb_len, 0);
  O3DX_HIP(hipGetLastError());
  G.view.skip_cells = w.d1;
  return 0;
}

static int64_t defer_cap(int64_t n) { return n / 4 + 64; }

static int normals_on_grid(GridBuild& G, const float* xyz, int64_t n, int mode, int knn, double radius,
                           const float* prior, float* out, float* kd2, void* ws, size_t ws_bytes, hipStream_t s) {
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  const int kneed = (int)std::min<int64_t>(knn, n);
  G.view.nbr = mode == O3DX_SEARCH_KNN ? debug_nbr(kneed, n) : nullptr;
  G.view.kd2 = mode == O3DX_SEARCH_KNN ? kd2 : nullptr;
  if (mode == O3DX_SEARCH_KNN && kneed >= 1 && !getenv("O3DX_NORMALS_TOPK")) {
    // LDS tiles (lane per query) -> wave per query -> exact register top-k,
    // each level serving the queries the previous one could not settle
    Arena ar((char*)ws + grid_ws_bytes(n), ws_bytes - grid_ws_bytes(n));
    int32_t* lens = ar.take<int32_t>(4);
    int32_t* list1 = ar.take<int32_t>(n);
    int32_t* list2 = ar.take<int32_t>(n);
    double* dmom = ar.take<double>(9 * defer_cap(n));
    int32_t* drow = ar.take<int32_t>(defer_cap(n));
    const int64_t upper = chunk_plan_upper(n, G.view, kTileQ);
    int32_t* chunks = ar.take<int32_t>(upper + 2);
    const size_t pws_bytes = chunk_plan_ws_bytes(n, (int64_t)G.view.ny * G.view.nz);
    void* pws = ar.take<char>(pws_bytes);
    O3DX_ARENA_CHECK(ar);
    O3DX_HIP(hipMemsetAsync(lens, 0, 4 * sizeof(int32_t), s));
    const bool tiles = !getenv("O3DX_NORMALS_NO_TILES");
    if (tiles) O3DX_TRY(chunk_plan(n, G.view, kTileQ, chunks, pws, pws_bytes, s));
    const int64_t nchunks = upper;
    KTimer kt("normals_knn", s);
    if (tiles && !getenv("O3DX_NESTED_OFF") && n >= 2 * kNestedMinQueries)
      O3DX_TRY(nested_tiles(G, n, kneed, occ_for(mode, knn), prior, out, list1, lens, ar, s));
    const int32_t* wl = tiles ? list1 : nullptr;
    const int32_t* wlen = tiles ? lens : nullptr;
    // the wave form grid-strides over its list (at most n queries)
    const unsigned gw = (unsigned)std::min<int64_t>((n + kWavesPerBlock - 1) / kWavesPerBlock, 8192);
    if (tiles) {
      // O3DX_TILE_DEBUG=1/2/3: stop after staging / histogram / list scan (profiling only; wrong normals)
      const char* dbg_env = getenv("O3DX_TILE_DEBUG");
      const int dbg = dbg_env ? atoi(dbg_env) : 0;
      KTimer kt_tile("normals_tile", s);
      if (kneed <= 32)
        hipLaunchKernelGGL(k_normals_knn_tile<32>, dim3((unsigned)nchunks), dim3(kTileQ), 0, s, G.view, chunks,
                           kneed, prior, out, list1, lens, dbg);
      else
        hipLaunchKernelGGL(k_normals_knn_tile<64>, dim3((unsigned)nchunks), dim3(kTileQ), 0, s, G.view, chunks,
                           kneed, prior, out, list1, lens, dbg);
    }
    {
      // the tiles hand on (almost only) queries whose k-th neighbour lies
      // beyond the shell-1 radius: start those at shell 2
      const int s0 = tiles ? 2 : 1;
      KTimer kt_wave("normals_wave", s);
      Deferred df;
      if (wl) {
        df.cap = defer_cap(n);
        df.mom = dmom;
        df.row = drow;
      }
      if (kneed <= 32)
        hipLaunchKernelGGL(k_normals_knn_wave<32>, dim3(gw), dim3(64 * kWavesPerBlock), 0, s, G.view, kneed, prior,
                           out, wl, wlen, list2, lens + 1, s0, df);
      else
        hipLaunchKernelGGL(k_normals_knn_wave<64>, dim3(gw), dim3(64 * kWavesPerBlock), 0, s, G.view, kneed, prior,
                           out, wl, wlen, list2, lens + 1, s0, df);
      if (df.cap)
        hipLaunchKernelGGL(k_finish_deferred, dim3(grid_for(std::min<int64_t>(n, df.cap), kBlock, 4096)), dim3(kBlock),
                           0, s, df, wlen, kneed, prior, out);
    }
    O3DX_DISPATCH_K(kneed, k_normals_knn, dim3(std::min(grid, 1024u)), dim3(kBlock), 0, s, G.view, xyz, kneed, 0,
                    radius, prior, out, list2, lens + 1);
  } else {
    KTimer kt("normals_knn", s);
    if (mode == O3DX_SEARCH_RADIUS)
      hipLaunchKernelGGL(k_normals_radius, dim3(grid), dim3(kBlock), 0, s, G.view, radius, prior, out);
    else
      O3DX_DISPATCH_K(kneed, k_normals_knn, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, kneed,
                      mode == O3DX_SEARCH_HYBRID ? 1 : 0, radius, prior, out, (const int32_t*)nullptr,
                      (const int32_t*)nullptr);
  }
  O3DX_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------ float64 clouds
// The float64 boundary (include/o3dx.h).  Open3D keeps points as float64
// (Vector3dVector, reference PointCloud.py:99-102) and computes kNN d^2 and
// the covariance moments on them; a float64 cloud that float32 cannot hold
// (LAS / E57 scans at georeferenced offsets, PointCloud.py:535-547, 646-687)
// must not be rounded.  The search frame is float32 p - o (o = the cloud's
// minimum bound, so the frame's magnitudes are the cloud's extent, and its
// rounding stays inside the grid's slack); every deciding d^2 and every
// moment comes from the exact float64 coordinates sorted alongside
// (GridView::pts64).

__global__ void __launch_bounds__(kBlock) k_proxy64(const double* __restrict__ xyz, int64_t n, double ox, double oy,
                                                    double oz, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    out[3 * i] = (float)(xyz[3 * i] - ox);
    out[3 * i + 1] = (float)(xyz[3 * i + 1] - oy);
    out[3 * i + 2] = (float)(xyz[3 * i + 2] - oz);
  }
}

// pts64[p] = the exact coordinates of sorted point p (w = original index)
__global__ void __launch_bounds__(kBlock) k_sort64(const float4* __restrict__ pts, int64_t n,
                                                   const double* __restrict__ xyz, double4* __restrict__ pts64) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int i = __float_as_int(pts[p].w);
    pts64[p] = make_double4(xyz[3 * (int64_t)i], xyz[3 * (int64_t)i + 1], xyz[3 * (int64_t)i + 2], (double)i);
  }
}

size_t grid64_ws_bytes(int64_t n, int cap_mult) {
  n = std::max<int64_t>(n, 1);
  return Arena::align(n * 3 * sizeof(float) + 1) + Arena::align(n * sizeof(double4) + 1) +
         Arena::align(aabb64_ws_bytes() + 64) + grid_ws_bytes(n, cap_mult) + 1024;
}

int grid64_build(const double* xyz, int64_t n, double target_occ, double min_h, void* ws, size_t ws_bytes,
                 hipStream_t s, GridBuild* out, const float* extra_src, int cap_mult, bool blocked,
                 const double* mm_host) {
  if (ws_bytes < grid64_ws_bytes(n, cap_mult)) return fail(O3DX_ENOMEM, "float64 grid workspace too small");
  Arena ar(ws, ws_bytes);
  float* proxy = ar.take<float>((size_t)std::max<int64_t>(n, 1) * 3);
  double4* pts64 = ar.take<double4>((size_t)std::max<int64_t>(n, 1));
  char* aws = ar.take<char>(aabb64_ws_bytes() + 64);
  const size_t gbytes = grid_ws_bytes(n, cap_mult);
  char* gws = ar.take<char>(gbytes);
  O3DX_ARENA_CHECK(ar);
  double mm[6] = {0, 0, 0, 0, 0, 0};
  if (mm_host) {
    std::memcpy(mm, mm_host, sizeof(mm));
  } else if (n > 0) {
    double* mmd = reinterpret_cast<double*>(aws + aabb64_ws_bytes());
    O3DX_TRY(aabb64_device(xyz, n, mmd, aws, s));
    O3DX_TRY(read_back(mm, mmd, sizeof(mm), s));
  }
  if (n > 0)
    hipLaunchKernelGGL(k_proxy64, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, mm[0], mm[1], mm[2],
                       proxy);
  O3DX_TRY(grid_build(proxy, n, target_occ, min_h, gws, gbytes, s, out, nullptr, extra_src, blocked, cap_mult));
  if (n > 0)
    hipLaunchKernelGGL(k_sort64, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, out->pts, n, xyz, pts64);
  O3DX_HIP(hipGetLastError());
  out->pts64 = pts64;
  out->view.pts64 = pts64;
  {
    // frame error: each frame coordinate (float)(p - o) lies in [0, extent],
    // rounded by at most half an ulp of the largest extent; a distance between
    // two frame points is then within 2 sqrt(3) of those of the exact one
    double fm = 0.0;
    for (int a = 0; a < 3; ++a) fm = std::max(fm, mm[3 + a] - mm[a]);
    const double half_ulp = fm > 0.0 ? std::ldexp(1.0, std::ilogb(fm) - 24) : 0.0;
    out->view.d64 = (float)(2.0 * std::sqrt(3.0) * half_ulp * 1.01 + 1e-30);
  }
  out->view.o64x = mm[0];
  out->view.o64y = mm[1];
  out->view.o64z = mm[2];
  return 0;
}

// Normals of a float64 cloud, a lane per point (sorted order): KNN / HYBRID
// through the register top-K in (d^2, index) order; RADIUS (every neighbour
// within r, sorted, Open3D's SearchRadius) read off in sorted pages of 32.
template <int K>
__device__ __forceinline__ void knn64_normal_query(const GridView& g, const double* __restrict__ xyz, int kneed,
                                                   int mode, double radius, const float* __restrict__ prior,
                                                   float* __restrict__ out, int64_t s) {
  const double4 q = g.pts64[s];
  const int oi = (int)q.w;
  MomAccSeq acc;
  acc.zero();
  int cnt = 0;
  if (mode == O3DX_SEARCH_RADIUS) {
    double lo_d = -1.0;
    int lo_i = -1;
    for (;;) {
      double bd[32];
      int bi[32];
      const int c = knn_search_dev64<32>(g, q.x, q.y, q.z, 32, true, radius, bd, bi, lo_d, lo_i);
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if (j < c) {
          const int64_t id = bi[j];
          acc.add(xyz[3 * id], xyz[3 * id + 1], xyz[3 * id + 2]);
        }
      cnt += c;
      if (c < 32) break;
      lo_d = bd[31];
      lo_i = bi[31];
    }
  } else {
    double bd[K];
    int bi[K];
    cnt = knn_search_dev64<K>(g, q.x, q.y, q.z, kneed, mode == O3DX_SEARCH_HYBRID, radius, bd, bi);
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (j < cnt) {
        const int id = bi[j];
        if (g.nbr && j < kneed) g.nbr[(int64_t)oi * kneed + j] = id;
        if (g.kd2 && j == cnt - 1) g.kd2[oi] = (float)(bd[j] * (1.0 + 1e-6));
        acc.add(xyz[3 * (int64_t)id], xyz[3 * (int64_t)id + 1], xyz[3 * (int64_t)id + 2]);
      }
  }
  finish_normal(cnt, acc, prior, oi, out);
}

// every point, a thread each (the round-5 launch form)
template <int K>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2))) k_normals_knn64(GridView g, const double* __restrict__ xyz, int kneed,
                                                          int mode, double radius, const float* __restrict__ prior,
                                                          float* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < g.n) knn64_normal_query<K>(g, xyz, kneed, mode, radius, prior, out, s);
}

// the sorted positions the float64 tiles handed on (*list_len of them)
template <int K>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2))) k_normals_knn64_list(GridView g, const double* __restrict__ xyz, int kneed,
                                                               int mode, double radius,
                                                               const float* __restrict__ prior,
                                                               float* __restrict__ out,
                                                               const int32_t* __restrict__ list,
                                                               const int32_t* __restrict__ list_len) {
  // a thread per listed query over a grid sized for the worst case (a
  // grid-stride loop here costs the query 36 more VGPRs: 1 wave per SIMD)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (int64_t)*list_len) knn64_normal_query<K>(g, xyz, kneed, mode, radius, prior, out, list[t]);
}

// The float64 tiles' hand-offs (KNN, kneed <= 32), a wave per query instead
// of a lane: each Chebyshev shell's rows (a face row = one point range, an
// inner row = its two end cells) become one flat candidate range spread over
// the 64 lanes, every lane keeping its own kW64Keep nearest in exact
// (d^2, index) order; the shell loop stops as knn_search_dev64's does (the
// k-th inside the shell's reach, counted conservatively over the lanes'
// lists).  The k nearest are then drawn from the lanes' heads in order — the
// same members in the same order as the lane form, accumulated in the same
// sequence (MomAccSeq).  A lane whose list runs dry while it saw more than it
// kept could hide a nearer one: such a query goes on to the lane form
// (fb list).  One lane form query walks its shells' candidates alone, one
// load batch at a time; here 64 lanes share them.
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
constexpr int kW64Keep = 8;
constexpr int kW64Waves = 4;
constexpr int kW64Cube = 0;  // (2: the radius-2 cube first — measured slower, 0.66 -> 0.74 ms)
// 4 waves per SIMD (128 VGPRs, a few spills): 0.74 -> 0.46 ms over 3 waves
// for the scan's 38K hand-offs (profiles/r06_f64_wave_ab.txt)
#ifndef O3DX_W64_WPE
#define O3DX_W64_WPE 4
#endif
#define O3DX_W64_ATTR __attribute__((amdgpu_waves_per_eu(O3DX_W64_WPE)))
__global__ void __launch_bounds__(64 * kW64Waves) O3DX_W64_ATTR k_normals_knn64_wave(GridView g, const double* __restrict__ xyz,
                                                                        int kneed, const float* __restrict__ prior,
                                                                        float* __restrict__ out,
                                                                        const int32_t* __restrict__ list,
                                                                        const int32_t* __restrict__ list_len,
                                                                        int32_t* __restrict__ fb,
                                                                        int32_t* __restrict__ fb_len, int keep_lim) {
  __shared__ int32_t s_a0[kW64Waves][64], s_l0[kW64Waves][64], s_a1[kW64Waves][64], s_rp[kW64Waves][65];
  __shared__ double s_md[kW64Waves][32];  // the members (want = min(kneed, seen) <= 32)
  __shared__ int32_t s_mi[kW64Waves][32];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t *ta0 = s_a0[wv], *tl0 = s_l0[wv], *ta1 = s_a1[wv], *trp = s_rp[wv];
  const int64_t m = *list_len;
  for (int64_t t = (int64_t)blockIdx.x * kW64Waves + wv; t < m; t += (int64_t)gridDim.x * kW64Waves) {
    const int64_t s = list[t];
    const double4 q = g.pts64[s];
    const int oi = (int)q.w;
    const double gqx = q.x - g.o64x, gqy = q.y - g.o64y, gqz = q.z - g.o64z;
    int cx, cy, cz;
    grid_cell(g, (float)gqx, (float)gqy, (float)gqz, cx, cy, cz);
    const int rmax = shell_rmax(g, cx, cy, cz);
    double bd[kW64Keep];
    int bi[kW64Keep];
#pragma unroll
    for (int j = 0; j < kW64Keep; ++j) {
      bd[j] = INFINITY;
      bi[j] = 0x7fffffff;
    }
    int seen = 0;
    // the first pass covers the whole cube of radius r0 (kW64Cube), then
    // shell by shell
    const int r0 = min(kW64Cube, rmax);
    for (int r = r0; r <= rmax; ++r) {
      const int side = 2 * r + 1, nrows = side * side;
      const bool cube = r == r0;
      for (int r0 = 0; r0 < nrows; r0 += 64) {
        const int row = r0 + lane;
        int a0 = 0, l0 = 0, a1 = 0, l1 = 0;
        if (row < nrows) {
          const int dz = row / side - r, dy = row % side - r;
          const int z = cz + dz, y = cy + dy;
          if (z >= 0 && z < g.nz && y >= 0 && y < g.ny) {
            const int rb = g.nx * (y + g.ny * z);
            if (cube || dz == -r || dz == r || dy == -r || dy == r) {  // a full row: the cells cx - r .. cx + r
              const int x0 = max(cx - r, 0), x1 = min(cx + r, g.nx - 1);
              if (x0 <= x1) {
                a0 = g.start[rb + x0];
                l0 = g.start[rb + x1 + 1] - a0;
              }
            } else {  // an inner row (r >= 1): its two end cells
              if (cx - r >= 0) {
                a0 = g.start[rb + cx - r];
                l0 = g.start[rb + cx - r + 1] - a0;
              }
              if (cx + r < g.nx) {
                a1 = g.start[rb + cx + r];
                l1 = g.start[rb + cx + r + 1] - a1;
              }
            }
          }
        }
        const int inc = wave_incl_scan(l0 + l1);
        const int tot = __shfl(inc, 63, 64);
        ta0[lane] = a0;
        tl0[lane] = l0;
        ta1[lane] = a1;
        trp[lane + 1] = inc;
        if (lane == 0) trp[0] = 0;
        wave_sync();
        int rw = 0;
        for (int b = 0; b < tot; b += 64) {
          const int f = b + lane;
          if (f < tot) {
            while (trp[rw + 1] <= f) ++rw;
            const int o = f - trp[rw];
            const int p = o < tl0[rw] ? ta0[rw] + o : ta1[rw] + (o - tl0[rw]);
            const double4 v = g.pts64[p];
            const double d = dist2_d4(q.x, q.y, q.z, v);
            const int id = (int)v.w;
            ++seen;
            if (lex_less(d, id, bd[kW64Keep - 1], bi[kW64Keep - 1])) {
#pragma unroll
              for (int j = kW64Keep - 1; j >= 0; --j) {
                const bool lt = lex_less(d, id, bd[j], bi[j]);
                const bool ltp = j > 0 ? lex_less(d, id, bd[j > 0 ? j - 1 : 0], bi[j > 0 ? j - 1 : 0]) : false;
                if (ltp) {
                  bd[j] = bd[j - 1];
                  bi[j] = bi[j - 1];
                } else if (lt) {
                  bd[j] = d;
                  bi[j] = id;
                }
              }
            }
          }
        }
        wave_sync();  // the row table is rewritten by the next 64 rows
      }
      const double B = cube_reach(g, gqx, gqy, gqz, cx, cy, cz, r) - g.slack;
      if (B > 0.0) {
        int c = 0;
#pragma unroll
        for (int j = 0; j < kW64Keep; ++j) c += bd[j] < B * B ? 1 : 0;
        if (wave_sum(c) >= kneed) break;  // the k-th lies inside the reach
      }
    }
    const int total = wave_sum(seen);
    const int want = min(kneed, total);
    // keep_lim < kW64Keep (tests of the hand-on): the lists as if shorter
#pragma unroll
    for (int e = 0; e < kW64Keep; ++e)
      if (e >= keep_lim) {
        bd[e] = INFINITY;
        bi[e] = 0x7fffffff;
      }
    const int kept = min(seen, keep_lim);
    // the want-th smallest d^2 over the lanes' lists: a bitwise search on the
    // (order-preserving) bits of the non-negative doubles, counted by ballots
    uint64_t kb = 0;
    for (int b = 62; b >= 0; --b) {
      const uint64_t t = kb | (1ull << b);
      int c = 0;
#pragma unroll
      for (int e = 0; e < kW64Keep; ++e) c += __popcll(__ballot((uint64_t)__double_as_longlong(bd[e]) < t));
      if (c < want) kb = t;
    }
    const double kd = __longlong_as_double((long long)kb);
    // members: d^2 < kd, then the smallest indices among d^2 == kd
    int lt = 0, eq = 0;
#pragma unroll
    for (int e = 0; e < kW64Keep; ++e) {
      lt += __popcll(__ballot(bd[e] < kd));
      eq += __popcll(__ballot(bd[e] == kd));
    }
    int ki = 0x7fffffff;  // the largest member index at d^2 == kd
    if (want > 0 && eq > want - lt) {  // an exact tie at the want-th distance
      int r = 0;
      for (int b = 30; b >= 0; --b) {
        const int t = r | (1 << b);
        int c = 0;
#pragma unroll
        for (int e = 0; e < kW64Keep; ++e) c += __popcll(__ballot(bd[e] == kd && bi[e] < t));
        if (c < want - lt) r = t;
      }
      ki = r;
    }
    // a lane that saw more than it kept hides candidates after its last kept
    // one: a nearer one than the want-th could hide there when that last kept
    // one is itself a member (keyed at or below (kd, ki))
    bool bad;
    {
      double ld = INFINITY;
      int li = 0x7fffffff;
#pragma unroll
      for (int e = 0; e < kW64Keep; ++e)
        if (e == kept - 1) {  // (no dynamic register index)
          ld = bd[e];
          li = bi[e];
        }
      bad = want > 0 && __any(seen > kept && kept > 0 && !lex_less(kd, ki, ld, li));
    }
    MomAccSeq acc;
    acc.zero();
    if (!bad && want > 0) {
      // compact the members into the wave's LDS rows, then rank them by
      // (d^2, index): member l lands in slot rank(l)
      double* md = s_md[wv];
      int32_t* mi = s_mi[wv];
      int base = 0;
#pragma unroll
      for (int e = 0; e < kW64Keep; ++e) {
        const bool mem = bd[e] < kd || (bd[e] == kd && bi[e] <= ki);
        const uint64_t mask = __ballot(mem);
        if (mem) {
          const int at = base + lanes_below(mask);
          md[at] = bd[e];
          mi[at] = bi[e];
        }
        base += __popcll(mask);
      }
      wave_sync();
      double myd = 0.0;
      int myi = 0, rank = 0;
      if (lane < want) {
        myd = md[lane];
        myi = mi[lane];
        for (int u = 0; u < want; ++u) rank += lex_less(md[u], mi[u], myd, myi) ? 1 : 0;
      }
      wave_sync();
      if (lane < want) mi[rank] = myi;
      wave_sync();
      // member l's coordinates, all loads at once; then Open3D's sequence
      double px = 0.0, py = 0.0, pz = 0.0;
      int id = 0;
      if (lane < want) {
        id = mi[lane];
        px = xyz[3 * (int64_t)id];
        py = xyz[3 * (int64_t)id + 1];
        pz = xyz[3 * (int64_t)id + 2];
        if (g.nbr) g.nbr[(int64_t)oi * kneed + lane] = id;
      }
      for (int u = 0; u < want; ++u) acc.add(readlane_f64(px, u), readlane_f64(py, u), readlane_f64(pz, u));
      wave_sync();
    }
    if (lane == 0) {
      if (bad) {
        fb[atomicAdd(fb_len, 1)] = (int32_t)s;
      } else {
        if (g.kd2 && want > 0) g.kd2[oi] = (float)(kd * (1.0 + 1e-6));
        finish_normal(want, acc, prior, oi, out);
      }
    }
  }
}

template <int K>
__global__ void __launch_bounds__(kBlock) k_knn_query64(GridView g, const double* __restrict__ q, int64_t nq,
                                                        int kneed, int hybrid, double radius, int kout,
                                                        int32_t* __restrict__ idx_out, double* __restrict__ d2_out,
                                                        int32_t* __restrict__ cnt_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  double bd[K];
  int bi[K];
  const int cnt = knn_search_dev64<K>(g, q[3 * i], q[3 * i + 1], q[3 * i + 2], kneed, hybrid != 0, radius, bd, bi);
  cnt_out[i] = cnt;
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (j < kout) {
      idx_out[i * kout + j] = j < cnt ? bi[j] : -1;
      if (d2_out) d2_out[i * kout + j] = j < cnt ? bd[j] : INFINITY;
    }
}

}  // namespace o3dx

using namespace o3dx;

extern "C" int o3dx_set_search_stats(int enable) {
  if (enable && !g_stats) {
    if (hipMalloc(&g_stats, 8 * sizeof(unsigned long long)) != hipSuccess) {
      g_stats = nullptr;
      return fail(O3DX_EIO, "stats buffer allocation failed");
    }
  }
  g_stats_on = enable != 0;
  if (g_stats && hipMemset(g_stats, 0, 8 * sizeof(unsigned long long)) != hipSuccess)
    return fail(O3DX_EIO, "stats reset failed");
  return 0;
}

extern "C" int o3dx_search_stats(int64_t* out) {
  if (!out) return fail(O3DX_EINVAL, "o3dx_search_stats: null output");
  unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g_stats && hipDeviceSynchronize() == hipSuccess)
    (void)hipMemcpy(v, g_stats, sizeof(v), hipMemcpyDeviceToHost);
  for (int i = 0; i < 8; ++i) out[i] = (int64_t)v[i];
  return 0;
}

extern "C" int o3dx_set_debug_neighbors(int32_t* buf, int64_t rows, int k) {
  if (buf && (rows < 0 || k < 1 || k > O3DX_MAX_KNN)) return fail(O3DX_EINVAL, "o3dx_set_debug_neighbors: bad k/rows");
  g_dbg_nbr = buf;
  g_dbg_rows = buf ? rows : 0;
  g_dbg_k = buf ? k : 0;
  return 0;
}

__global__ void __launch_bounds__(kBlock) k_fast_eigen(const double* __restrict__ cov, int64_t m,
                                                       double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double c[6], v[3];
  for (int j = 0; j < 6; ++j) c[j] = cov[6 * i + j];
  fast_eigen3x3(c, v);
  for (int j = 0; j < 3; ++j) out[3 * i + j] = v[j];
}

__global__ void __launch_bounds__(kBlock) k_libm_probe(const double* __restrict__ x, int64_t n, int fn,
                                                       double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  out[i] = fn == 0 ? acos(v) : fn == 1 ? cos(v) : sqrt(v);
}

extern "C" int o3dx_fast_eigen3x3(const double* cov, int64_t m, double* out, void* stream) {
  if (m < 0 || (m > 0 && (!cov || !out))) return fail(O3DX_EINVAL, "o3dx_fast_eigen3x3: bad arguments");
  if (m == 0) return 0;
  hipLaunchKernelGGL(k_fast_eigen, dim3((unsigned)((m + kBlock - 1) / kBlock)), dim3(kBlock), 0, as_stream(stream),
                     cov, m, out);
  O3DX_HIP(hipGetLastError());
  return 0;
}

extern "C" int o3dx_libm_probe(const double* x, int64_t n, int fn, double* out, void* stream) {
  if (n < 0 || fn < 0 || fn > 2 || (n > 0 && (!x || !out))) return fail(O3DX_EINVAL, "o3dx_libm_probe: bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_libm_probe, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, as_stream(stream), x,
                     n, fn, out);
  O3DX_HIP(hipGetLastError());
  return 0;
}

extern "C" size_t o3dx_normals_workspace_bytes(int64_t n) {
  n = std::max<int64_t>(n, 1);
  // grid rows (ny * nz) are bounded by the cell cap
  const int64_t rows = cap_cells(n, 4);
  return grid_ws_bytes(n) + 3 * Arena::align((n + 3) * 4) + Arena::align((n / 64 + rows + 4) * 4) +
         chunk_plan_ws_bytes(n, rows) + nested_ws_bytes(n) + Arena::align(9 * 8 * defer_cap(n) + 1) +
         Arena::align(4 * defer_cap(n) + 1) + 4096;
}

extern "C" int o3dx_estimate_normals(const float* xyz, int64_t n, int mode, int knn, double radius,
                                     const float* prior, float* out, float* kd2, void* ws, size_t ws_bytes,
                                     void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !out))) return fail(O3DX_EINVAL, "o3dx_estimate_normals: bad arguments");
  if (mode != O3DX_SEARCH_KNN && mode != O3DX_SEARCH_RADIUS && mode != O3DX_SEARCH_HYBRID)
    return fail(O3DX_EINVAL, "o3dx_estimate_normals: unknown search mode %d", mode);
  if (mode != O3DX_SEARCH_RADIUS && (knn < 0 || knn > O3DX_MAX_KNN))
    return fail(O3DX_ENOTSUP, "knn/max_nn %d outside [0, %d]", knn, O3DX_MAX_KNN);
  if (mode != O3DX_SEARCH_KNN && !(radius > 0.0)) return fail(O3DX_EINVAL, "radius must be > 0");
  if (!ws || ws_bytes < o3dx_normals_workspace_bytes(n)) return fail(O3DX_ENOMEM, "normals workspace too small");
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  GridBuild G;
  O3DX_TRY(grid_build(xyz, n, occ_for(mode, knn), 0.0, ws, ws_bytes, s, &G));
  return normals_on_grid(G, xyz, n, mode, knn, radius, prior, out, kd2, ws, ws_bytes, s);
}

extern "C" int o3dx_estimate_normals_voxel(const double* geom, const float* voxel_pts, const float* xyz, int64_t n,
                                           int mode, int knn, double radius, const float* prior, float* out,
                                           float* kd2, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !out || !geom))) return fail(O3DX_EINVAL, "o3dx_estimate_normals_voxel: bad arguments");
  if (mode != O3DX_SEARCH_KNN && mode != O3DX_SEARCH_RADIUS && mode != O3DX_SEARCH_HYBRID)
    return fail(O3DX_EINVAL, "o3dx_estimate_normals_voxel: unknown search mode %d", mode);
  if (mode != O3DX_SEARCH_RADIUS && (knn < 0 || knn > O3DX_MAX_KNN))
    return fail(O3DX_ENOTSUP, "knn/max_nn %d outside [0, %d]", knn, O3DX_MAX_KNN);
  if (mode != O3DX_SEARCH_KNN && !(radius > 0.0)) return fail(O3DX_EINVAL, "radius must be > 0");
  if (!ws || ws_bytes < o3dx_normals_workspace_bytes(n)) return fail(O3DX_ENOMEM, "normals workspace too small");
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  const int rd = normals_dense_vox(geom, reinterpret_cast<const float4*>(voxel_pts), xyz, n, mode, knn, prior, out,
                                   kd2, ws, ws_bytes, s);
  if (rd != 1) return rd;
  GridBuild G;
  const int rc = grid_from_voxels(geom, reinterpret_cast<const float4*>(voxel_pts), n, occ_for(mode, knn), ws, ws_bytes,
                                  s, &G);
  if (rc == 1) O3DX_TRY(grid_build(xyz, n, occ_for(mode, knn), 0.0, ws, ws_bytes, s, &G));  // no usable voxel grid
  else if (rc != 0) return rc;
  return normals_on_grid(G, xyz, n, mode, knn, radius, prior, out, kd2, ws, ws_bytes, s);
}

extern "C" size_t o3dx_knn_workspace_bytes(int64_t n) { return grid_ws_bytes(n) + 1024; }

extern "C" int o3dx_knn_search(const float* xyz, int64_t n, const float* queries, int64_t nq, int mode, int knn,
                               double radius, int32_t* idx_out, double* d2_out, int32_t* cnt_out, void* ws,
                               size_t ws_bytes, void* stream) {
  if (n < 0 || nq < 0 || (n > 0 && !xyz) || (nq > 0 && (!queries || !idx_out || !cnt_out)))
    return fail(O3DX_EINVAL, "o3dx_knn_search: bad arguments");
  if (mode == O3DX_SEARCH_RADIUS)
    return fail(O3DX_ENOTSUP, "o3dx_knn_search: radius mode needs a variable-length result (use HYBRID)");
  if (mode != O3DX_SEARCH_KNN && mode != O3DX_SEARCH_HYBRID) return fail(O3DX_EINVAL, "unknown search mode");
  if (knn < 1 || knn > O3DX_MAX_KNN) return fail(O3DX_ENOTSUP, "knn %d outside [1, %d]", knn, O3DX_MAX_KNN);
  if (!ws || ws_bytes < o3dx_knn_workspace_bytes(n)) return fail(O3DX_ENOMEM, "knn workspace too small");
  if (nq == 0) return 0;
  hipStream_t s = as_stream(stream);
  GridBuild G;
  O3DX_TRY(grid_build(xyz, n, occ_for(mode, knn), 0.0, ws, ws_bytes, s, &G));
  const int kneed = (int)std::min<int64_t>(knn, n);
  const unsigned grid = (unsigned)((nq + kBlock - 1) / kBlock);
  O3DX_DISPATCH_K(knn, k_knn_query, dim3(grid), dim3(kBlock), 0, s, G.view, queries, nq, kneed,
                  mode == O3DX_SEARCH_HYBRID ? 1 : 0, radius, knn, idx_out, d2_out, cnt_out);
  O3DX_HIP(hipGetLastError());
  return 0;
}

// -------------------------------------------- voxel_down_sample + normals
// The pipeline pcd.voxel_down_sample(vs).estimate_normals(KNN) (reference
// PointCloud.py:361, :68) in one call: the normals kernels over the kept
// voxel table are queued right behind the voxel kernels, before the host reads
// the representative count back (their grids and lists do not need it), so
// the GPU never idles between the two; once the counts are known the
// applicability test of the table path is replayed, and when it fails the
// normals are recomputed by o3dx_estimate_normals_voxel's general path.
namespace o3dx {
struct SpecNormals {
  const float* rep_xyz;
  int64_t ncap;
  int knn;
  float* out;
  void* ws;
  size_t ws_bytes;
  hipStream_t s;
  bool launched;
  bool lens_zeroed;  // the normals' hand-off counters (ws head) cleared by the bounds pass
};
static int spec_normals_hook(void* ctx, const double* geom, const void* vox) {
  SpecNormals& c = *static_cast<SpecNormals*>(ctx);
  const int rc = normals_dense_vox(geom, static_cast<const float4*>(vox), c.rep_xyz, c.ncap, O3DX_SEARCH_KNN, c.knn,
                                   nullptr, c.out, nullptr, c.ws, c.ws_bytes, c.s, true, c.lens_zeroed);
  c.launched = rc == 0;
  return rc == 1 ? 0 : rc;
}
}  // namespace o3dx

extern "C" int o3dx_voxel_down_sample_normals(const float* xyz, int64_t n, const double* min_bound,
                                              const double* max_bound, double voxel_size, int knn, int32_t* rep_idx,
                                              float* rep_xyz, float* normals, int64_t* m_host, float* voxel_pts,
                                              int64_t voxel_cells, double* geom, void* ws, size_t ws_bytes, void* nws,
                                              size_t nws_bytes, void* stream) {
  if (!rep_xyz || !normals || !voxel_pts || !geom || !nws || nws_bytes < o3dx_normals_workspace_bytes(n))
    return fail(O3DX_EINVAL, "o3dx_voxel_down_sample_normals: bad arguments");
  if (knn < 0 || knn > O3DX_MAX_KNN) return fail(O3DX_ENOTSUP, "knn %d outside [0, %d]", knn, O3DX_MAX_KNN);
  SpecNormals c{rep_xyz, n, knn, normals, nws, nws_bytes, as_stream(stream), false, true};
  // normals_dense_vox's hand-off counters: the first 16 B of its workspace
  O3DX_TRY(voxel_down_sample_hooked(xyz, n, min_bound, max_bound, voxel_size, rep_idx, rep_xyz, m_host, voxel_pts,
                                    voxel_cells, geom, ws, ws_bytes, stream, spec_normals_hook, &c,
                                    ZeroSpan{static_cast<uint8_t*>(nws), 4 * sizeof(int32_t)}));
  const int64_t m = *m_host;
  double kth;
  if (c.launched && geom[10] == 0.0 && dense_vox_applicable(geom, reinterpret_cast<const float4*>(voxel_pts), m, O3DX_SEARCH_KNN, knn,
                                         &kth) &&
      std::min<int64_t>(knn, m) == knn)
    return 0;
  return o3dx_estimate_normals_voxel(geom, voxel_pts, rep_xyz, m, O3DX_SEARCH_KNN, knn, 0.0, nullptr, normals, nullptr,
                                     nws, nws_bytes, stream);
}

// ------------------------------------------------------ float64 boundary
// [float64 grid][tiles: lens, hand-off list, chunk starts, chunk-plan scratch,
// the wave form's hand-off list]
static size_t normals64_tiles_bytes(int64_t n) {
  n = std::max<int64_t>(n, 1);
  const int64_t rows = cap_cells(n, 4);  // grid rows (ny * nz) are bounded by the cell cap
  return Arena::align(4 * 4 + 1) + 2 * Arena::align(n * 4 + 1) + Arena::align((n / 64 + rows + 4) * 4 + 1) +
         chunk_plan_ws_bytes(n, rows) + 1024;
}
extern "C" size_t o3dx_normals_f64_workspace_bytes(int64_t n) {
  return grid64_ws_bytes(n) + normals64_tiles_bytes(n) + 1024;
}

extern "C" int o3dx_estimate_normals_f64(const double* xyz, int64_t n, int mode, int knn, double radius,
                                         const float* prior, float* out, float* kd2, void* ws, size_t ws_bytes,
                                         void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !out))) return fail(O3DX_EINVAL, "o3dx_estimate_normals_f64: bad arguments");
  if (mode != O3DX_SEARCH_KNN && mode != O3DX_SEARCH_RADIUS && mode != O3DX_SEARCH_HYBRID)
    return fail(O3DX_EINVAL, "o3dx_estimate_normals_f64: unknown search mode %d", mode);
  if (mode != O3DX_SEARCH_RADIUS && (knn < 0 || knn > O3DX_MAX_KNN))
    return fail(O3DX_ENOTSUP, "knn/max_nn %d outside [0, %d]", knn, O3DX_MAX_KNN);
  if (mode != O3DX_SEARCH_KNN && !(radius > 0.0)) return fail(O3DX_EINVAL, "radius must be > 0");
  if (!ws || ws_bytes < o3dx_normals_f64_workspace_bytes(n)) return fail(O3DX_ENOMEM, "normals workspace too small");
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  GridBuild G;
  O3DX_TRY(grid64_build(xyz, n, occ_for(mode, knn), 0.0, ws, ws_bytes, s, &G));
  const int kneed = (int)std::min<int64_t>(knn, n);
  G.view.nbr = mode == O3DX_SEARCH_KNN ? debug_nbr(kneed, n) : nullptr;
  G.view.kd2 = mode == O3DX_SEARCH_KNN ? kd2 : nullptr;
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  KTimer kt("normals_f64", s);
  if (mode == O3DX_SEARCH_KNN && kneed >= 1 && kneed <= 32 && !getenv("O3DX_F64_NO_TILES")) {
    // LDS tiles on the float32 frame, the exact float64 order deciding
    // (k_normals_knn_tile<32, *, true>), then the lane-per-query form for the
    // queries they hand on
    const size_t g64 = grid64_ws_bytes(n);
    G.view.xyz64 = xyz;
    Arena ar((char*)ws + g64, ws_bytes - g64);
    int32_t* lens = ar.take<int32_t>(4);
    int32_t* list = ar.take<int32_t>(n);
    const int64_t upper = chunk_plan_upper(n, G.view, kTileQ);
    int32_t* chunks = ar.take<int32_t>(upper + 2);
    const size_t pws_bytes = chunk_plan_ws_bytes(n, (int64_t)G.view.ny * G.view.nz);
    void* pws = ar.take<char>(pws_bytes);
    int32_t* list2 = ar.take<int32_t>(n);
    O3DX_ARENA_CHECK(ar);
    O3DX_HIP(hipMemsetAsync(lens, 0, 4 * sizeof(int32_t), s));
    O3DX_TRY(chunk_plan(n, G.view, kTileQ, chunks, pws, pws_bytes, s));
    {
      KTimer kt_tile("normals_tile64", s);
      hipLaunchKernelGGL((k_normals_knn_tile<32, MomAccA, true>), dim3((unsigned)upper), dim3(kTileQ), 0, s, G.view,
                         chunks, kneed, prior, out, list, lens, 0);
    }
    if (getenv("O3DX_F64_NO_WAVE")) {  // every hand-off to the lane form (A/B, tests)
      O3DX_DISPATCH_K(kneed, k_normals_knn64_list, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, kneed, mode, radius,
                      prior, out, (const int32_t*)list, (const int32_t*)lens);
    } else {
      // the hand-offs a wave each; the few it cannot settle (lens[2]) to the lane form
      KTimer kt_wave("normals_wave64", s);
      const unsigned wblocks = (unsigned)std::min<int64_t>((n + kW64Waves - 1) / kW64Waves, 2048);
      const char* kl = getenv("O3DX_F64_WAVE_KEEP");  // tests: a shorter list hands more queries on
      const int keep = kl ? std::max(1, std::min(kW64Keep, atoi(kl))) : kW64Keep;
      hipLaunchKernelGGL(k_normals_knn64_wave, dim3(wblocks), dim3(64 * kW64Waves), 0, s, G.view, xyz, kneed, prior,
                         out, (const int32_t*)list, (const int32_t*)lens, list2, lens + 2, keep);
      kt_wave.stop();
      O3DX_DISPATCH_K(kneed, k_normals_knn64_list, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, kneed, mode, radius,
                      prior, out, (const int32_t*)list2, (const int32_t*)(lens + 2));
    }
  } else if (mode == O3DX_SEARCH_RADIUS) {
    hipLaunchKernelGGL(k_normals_knn64<4>, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, 0, mode, radius, prior, out);
  } else {
    O3DX_DISPATCH_K(kneed, k_normals_knn64, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, kneed, mode, radius, prior,
                    out);
  }
  O3DX_HIP(hipGetLastError());
  return 0;
}

extern "C" size_t o3dx_knn_f64_workspace_bytes(int64_t n) { return grid64_ws_bytes(n) + 1024; }

extern "C" int o3dx_knn_search_f64(const double* xyz, int64_t n, const double* queries, int64_t nq, int mode, int knn,
                                   double radius, int32_t* idx_out, double* d2_out, int32_t* cnt_out, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (n < 0 || nq < 0 || (n > 0 && !xyz) || (nq > 0 && (!queries || !idx_out || !cnt_out)))
    return fail(O3DX_EINVAL, "o3dx_knn_search_f64: bad arguments");
  if (mode == O3DX_SEARCH_RADIUS)
    return fail(O3DX_ENOTSUP, "o3dx_knn_search_f64: radius mode needs a variable-length result (use HYBRID)");
  if (mode != O3DX_SEARCH_KNN && mode != O3DX_SEARCH_HYBRID) return fail(O3DX_EINVAL, "unknown search mode");
  if (knn < 1 || knn > O3DX_MAX_KNN) return fail(O3DX_ENOTSUP, "knn %d outside [1, %d]", knn, O3DX_MAX_KNN);
  if (!ws || ws_bytes < o3dx_knn_f64_workspace_bytes(n)) return fail(O3DX_ENOMEM, "knn workspace too small");
  if (nq == 0) return 0;
  hipStream_t s = as_stream(stream);
  GridBuild G;
  O3DX_TRY(grid64_build(xyz, n, occ_for(mode, knn), 0.0, ws, ws_bytes, s, &G));
  const int kneed = (int)std::min<int64_t>(knn, n);
  const unsigned grid = (unsigned)((nq + kBlock - 1) / kBlock);
  O3DX_DISPATCH_K(knn, k_knn_query64, dim3(grid), dim3(kBlock), 0, s, G.view, queries, nq, kneed,
                  mode == O3DX_SEARCH_HYBRID ? 1 : 0, radius, knn, idx_out, d2_out, cnt_out);
  O3DX_HIP(hipGetLastError());
  return 0;
}
