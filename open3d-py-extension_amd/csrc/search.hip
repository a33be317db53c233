// search.hip — one KDTreeFlann query of any size on the device.
//
// Replaces KDTreeFlann.search_knn_vector_3d / search_radius_vector_3d /
// search_hybrid_vector_3d behind the reference's get_points_by_knn /
// get_points_radius (reference open3dpypro/PointCloud.py:148-163), whose
// defaults ask for up to 10^6 neighbours (max_nn = 1000000) or a 30-unit
// radius — sizes the register top-k of the batched search (<= O3DX_MAX_KNN)
// does not serve.  One query, so the work is a streaming pass over the cloud:
//   1. d^2 of every point in float64, nanoflann's order ((dx dx + dy dy) +
//      dz dz) on the cloud's own coordinates (float32 values upcast exactly,
//      or the float64 boundary's float64 values);
//   2. the candidates: d^2 < r^2 (radius / hybrid), or — kNN — the points
//      whose d^2 key falls in the histogram bins up to the one holding the
//      k-th (8192 bins on the float64 key's exponent and top mantissa bits,
//      a quarter octave each), compacted in ascending index order;
//   3. a stable radix sort of the candidates by d^2 (rocPRIM), so equal
//      distances keep ascending index: the (d^2, index) order of the
//      oracle; the first k (or all within the radius) are the result.
#include <hipcub/hipcub.hpp>
#include <vector>

#include "common.hpp"

namespace o3dx {

constexpr int kSelBits = 13;                 // histogram bins: d^2 key bits [62 - 13 + 1, 62]
constexpr int kSelShift = 63 - kSelBits;     // 50
constexpr int kSelBins = 1 << kSelBits;      // 8192 (32 KB of LDS)
constexpr int kSelBlocks = 1024;

__device__ __forceinline__ uint64_t d2_key(double d2) { return (uint64_t)__double_as_longlong(d2); }

template <class T>
__global__ void __launch_bounds__(kBlock) k_search_d2(const T* __restrict__ xyz, int64_t n, double qx, double qy,
                                                      double qz, double r2, uint64_t* __restrict__ key,
                                                      uint8_t* __restrict__ flag, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kSelBins];
  if (hist)
    for (int t = threadIdx.x; t < kSelBins; t += kBlock) h[t] = 0u;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double dx = qx - (double)xyz[3 * i], dy = qy - (double)xyz[3 * i + 1], dz = qz - (double)xyz[3 * i + 2];
    double d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    const bool in = d < r2;  // NaN coordinates: never a neighbour
    const uint64_t k = d2_key(d);
    key[i] = k;
    flag[i] = in ? 1 : 0;
    if (hist && in) atomicAdd(&h[(int)(k >> kSelShift)], 1u);
  }
  __syncthreads();
  if (hist)
    for (int t = threadIdx.x; t < kSelBins; t += kBlock)
      if (h[t]) atomicAdd(&hist[t], h[t]);
}

// kNN: candidates = keys in the bins up to kth_bin (flag rewritten)
__global__ void __launch_bounds__(kBlock) k_search_cut(const uint64_t* __restrict__ key, int64_t n, uint64_t key_lim,
                                                       uint8_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = (flag[i] && key[i] < key_lim) ? 1 : 0;
}

__global__ void __launch_bounds__(kBlock) k_search_gather(const uint64_t* __restrict__ key,
                                                          const int32_t* __restrict__ idx,
                                                          const int64_t* __restrict__ count,
                                                          uint64_t* __restrict__ ckey) {
  const int64_t m = *count;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
    ckey[j] = key[idx[j]];
}

__global__ void __launch_bounds__(kBlock) k_search_emit(const uint64_t* __restrict__ skey,
                                                        const int32_t* __restrict__ sidx, int64_t m,
                                                        int32_t* __restrict__ idx_out, double* __restrict__ d2_out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    idx_out[j] = sidx[j];
    if (d2_out) d2_out[j] = __longlong_as_double((long long)skey[j]);
  }
}

struct SearchWs {
  uint64_t *key, *ckey, *skey;
  int32_t *idx, *sidx, *scan_tmp;
  uint8_t* flag;
  uint32_t* hist;
  int64_t* count;
  void* sort_tmp;
  size_t sort_bytes;
};

// Stable radix sort of (cell key, point index) pairs for grid_build's
// large cell arrays (grid.hip): keys below 2^bits.
size_t cell_sort_temp_bytes(int64_t n, int bits) {
  size_t b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const int32_t*)nullptr, (int32_t*)nullptr, (int)std::max<int64_t>(n, 1), 0,
                                           bits);
  return b;
}

int cell_sort(const uint32_t* key, uint32_t* skey, const int32_t* val, int32_t* sval, int64_t n, int bits, void* tmp,
              size_t tmp_bytes, hipStream_t s) {
  O3DX_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, key, skey, val, sval, (int)n, 0, bits, s));
  return 0;
}

static size_t sort_temp_bytes(int64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, std::max<int64_t>(n, 1), 0, 63);
  return b;
}

static size_t search_carve(Arena& ar, int64_t n, SearchWs* w) {
  n = std::max<int64_t>(n, 1);
  w->key = ar.take<uint64_t>(n);
  w->ckey = ar.take<uint64_t>(n);
  w->skey = ar.take<uint64_t>(n);
  w->idx = ar.take<int32_t>(n);
  w->sidx = ar.take<int32_t>(n);
  w->scan_tmp = ar.take<int32_t>(compact_workspace_ints(n));
  w->flag = ar.take<uint8_t>(n + 16);
  w->hist = ar.take<uint32_t>(kSelBins);
  w->count = ar.take<int64_t>(2);
  w->sort_bytes = sort_temp_bytes(n);
  w->sort_tmp = ar.take<char>(w->sort_bytes);
  return ar.used;
}

template <class T>
static int search_one(const T* xyz, int64_t n, const double* q, int mode, int64_t knn, double radius, int32_t* idx_out,
                      double* d2_out, int64_t cap, int64_t* count_host, void* ws, size_t ws_bytes, hipStream_t s) {
  Arena ar(ws, ws_bytes);
  SearchWs w;
  search_carve(ar, n, &w);
  O3DX_ARENA_CHECK(ar);
  *count_host = 0;
  if (n == 0 || (mode != O3DX_SEARCH_RADIUS && knn <= 0)) return 0;
  const bool use_r = mode != O3DX_SEARCH_KNN;
  const double r2 = use_r ? radius * radius : INFINITY;
  const bool sel = mode != O3DX_SEARCH_RADIUS;  // the k nearest (of those within r for hybrid)
  if (sel) O3DX_HIP(hipMemsetAsync(w.hist, 0, kSelBins * sizeof(uint32_t), s));
  const unsigned g = grid_for(n, kBlock, kSelBlocks);
  KTimer kt("search_one", s);
  hipLaunchKernelGGL(k_search_d2<T>, dim3(g), dim3(kBlock), 0, s, xyz, n, q[0], q[1], q[2], r2, w.key, w.flag,
                     sel ? w.hist : nullptr);
  if (sel) {
    // the bin of the k-th smallest key: everything below it is in, it is cut
    // at its upper edge (a quarter octave of d^2 holds few points past the k-th)
    std::vector<uint32_t> h(kSelBins);
    O3DX_TRY(read_back(h.data(), w.hist, kSelBins * sizeof(uint32_t), s));
    int64_t cum = 0;
    int b = kSelBins - 1;
    for (int i = 0; i < kSelBins; ++i) {
      cum += h[i];
      if (cum >= knn) {
        b = i;
        break;
      }
    }
    if (cum >= knn && b < kSelBins - 1)
      hipLaunchKernelGGL(k_search_cut, dim3(g), dim3(kBlock), 0, s, w.key, n, (uint64_t)(b + 1) << kSelShift, w.flag);
  }
  O3DX_TRY(compact_flags(w.flag, n, w.idx, nullptr, w.count, w.scan_tmp, s));
  int64_t m = 0;
  O3DX_TRY(read_back(&m, w.count, sizeof(int64_t), s));
  if (m == 0) return 0;
  hipLaunchKernelGGL(k_search_gather, dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, w.key, w.idx, w.count,
                     w.ckey);
  size_t sb = w.sort_bytes;
  // stable: equal d^2 keep the compaction's ascending index
  O3DX_HIP(hipcub::DeviceRadixSort::SortPairs(w.sort_tmp, sb, w.ckey, w.skey, w.idx, w.sidx, m, 0, 63, s));
  const int64_t k = sel ? std::min<int64_t>(m, knn) : m;
  const int64_t put = std::min<int64_t>(k, cap);
  if (put > 0)
    hipLaunchKernelGGL(k_search_emit, dim3(grid_for(put, kBlock, 8192)), dim3(kBlock), 0, s, w.skey, w.sidx, put,
                       idx_out, d2_out);
  O3DX_HIP(hipGetLastError());
  O3DX_HIP(hipStreamSynchronize(s));
  *count_host = k;
  return 0;
}

}  // namespace o3dx

using namespace o3dx;

extern "C" size_t o3dx_search_one_workspace_bytes(int64_t n) {
  Arena ar(nullptr, 0);
  SearchWs w;
  return search_carve(ar, n, &w) + 1024;
}

extern "C" int o3dx_search_one(const void* xyz, int xyz_f64, int64_t n, const double* query_host, int mode,
                               int64_t knn, double radius, int32_t* idx_out, double* d2_out, int64_t cap,
                               int64_t* count_host, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || (n > 0 && !xyz) || !query_host || !count_host || cap < 0 || (cap > 0 && !idx_out))
    return fail(O3DX_EINVAL, "o3dx_search_one: bad arguments");
  if (mode != O3DX_SEARCH_KNN && mode != O3DX_SEARCH_RADIUS && mode != O3DX_SEARCH_HYBRID)
    return fail(O3DX_EINVAL, "o3dx_search_one: unknown search mode %d", mode);
  if (!ws || ws_bytes < o3dx_search_one_workspace_bytes(n))
    return fail(O3DX_ENOMEM, "o3dx_search_one: workspace too small");
  hipStream_t s = as_stream(stream);
  if (xyz_f64)
    return search_one(static_cast<const double*>(xyz), n, query_host, mode, knn, radius, idx_out, d2_out, cap,
                      count_host, ws, ws_bytes, s);
  return search_one(static_cast<const float*>(xyz), n, query_host, mode, knn, radius, idx_out, d2_out, cap, count_host,
                    ws, ws_bytes, s);
}
