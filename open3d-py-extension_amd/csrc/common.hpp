// common.hpp — shared host/device helpers of libo3dx (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/o3dx.h"

namespace o3dx {

// ------------------------------------------------------------------ errors
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define O3DX_HIP(call)                                                            \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess)                                                         \
      return ::o3dx::fail(O3DX_EIO, "%s:%d %s: %s", __FILE__, __LINE__, #call,    \
                          hipGetErrorString(e_));                                 \
  } while (0)

#define O3DX_TRY(expr)        \
  do {                        \
    int rc_ = (expr);         \
    if (rc_ != 0) return rc_; \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// --------------------------------------------------------------- workspace
// Bump allocator over the caller's scratch buffer (256-B aligned pieces).
struct Arena {
  char* base;
  size_t cap, used = 0;
  bool dry;  // dry run: only count bytes
  Arena(void* p, size_t bytes) : base((char*)p), cap(bytes), dry(p == nullptr) {}
  static size_t align(size_t b) { return (b + 255) & ~size_t(255); }
  template <class T>
  T* take(size_t count) {
    size_t b = align(count * sizeof(T) + 1);
    char* p = dry ? nullptr : base + used;
    used += b;
    return reinterpret_cast<T*>(p);
  }
  bool ok() const { return dry || used <= cap; }
};

#define O3DX_ARENA_CHECK(ar)                                                              \
  do {                                                                                    \
    if (!(ar).ok())                                                                       \
      return ::o3dx::fail(O3DX_ENOMEM, "workspace too small: need %zu bytes, have %zu", \
                          (ar).used, (ar).cap);                                           \
  } while (0)

// --------------------------------------------------------------- launching
constexpr int kBlock = 256;
inline unsigned grid_for(int64_t n, int block = kBlock, int64_t cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ----------------------------------------------------------- device utils
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

// Exclusive scan across a block of BLOCK threads (BLOCK multiple of 64).
// `sh` needs BLOCK/64 ints.  Returns the exclusive prefix, *total = block sum.
template <int BLOCK>
__device__ __forceinline__ int block_excl_scan(int v, int* sh, int* total) {
  const int w = threadIdx.x >> 6, l = lane_id();
  int inc = wave_incl_scan(v);
  if (l == 63) sh[w] = inc;
  __syncthreads();
  if (w == 0) {
    int s = (l < BLOCK / 64) ? sh[l] : 0;
    int si = wave_incl_scan(s);
    if (l < BLOCK / 64) sh[l] = si - s;
    if (l == BLOCK / 64 - 1) sh[BLOCK / 64] = si;
  }
  __syncthreads();
  int res = inc - v + sh[w];
  *total = sh[BLOCK / 64];
  __syncthreads();
  return res;
}

// Block reduction of a double (fixed order: wave xor-tree, then waves in order).
template <int BLOCK>
__device__ __forceinline__ double block_sum_f64(double v, double* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < BLOCK / 64; ++i) r += sh[i];
  __syncthreads();
  return r;  // valid in thread 0
}

// ---------------------------------------------------------- kernel timing
// RAII bracket of a launch with hipEvents on its stream (only when enabled by
// o3dx_set_kernel_timing); read back lazily by o3dx_kernel_timing.
bool timing_on();
bool timing_wanted(const char* name);
void timing_push(const char* name, hipEvent_t a, hipEvent_t b);
hipEvent_t timing_event();           // from the recycled pool (or new)
void timing_release(hipEvent_t e);   // back to the pool
// Wait for the stream's work to finish (polling first; see core.hip).
int host_wait(hipStream_t s);
// Device -> host copy of a small result, then host_wait.
int read_back(void* dst_host, const void* src_dev, size_t bytes, hipStream_t s);
int read_back_begin(const void* src_dev, size_t bytes, hipStream_t s);  // <= 64 KB, one pending per thread
int read_back_end(void* dst_host, size_t bytes);
struct KTimer {
  const char* name;
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  KTimer(const char* n, hipStream_t st) : name(n), s(st) {
    if (timing_wanted(n)) {
      a = timing_event();
      b = timing_event();
      if (a && b) {
        (void)hipEventRecord(a, s);
      } else {
        timing_release(a);
        timing_release(b);
        a = b = nullptr;
      }
    }
  }
  void stop() {
    if (a && b) {
      (void)hipEventRecord(b, s);
      timing_push(name, a, b);
    }
    a = b = nullptr;
  }
  void cancel() {  // drop without recording (a later KTimer of the same name takes over)
    timing_release(a);
    timing_release(b);
    a = b = nullptr;
  }
  ~KTimer() { stop(); }
};

// ---------------------------------------------------------- host helpers
// Exclusive scan of `n` int32 counts into `out` (n+1 entries, out[n] = total).
// Workspace: scan_workspace_ints(n) ints.
size_t scan_workspace_ints(int64_t n);
int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* tmp, hipStream_t s);

// Flag compaction: positions of set bytes, ascending.  `pos_out` (nullable)
// receives the exclusive prefix at every index; `idx_out` the compacted
// indices; *count_dev the total (device int64).
size_t compact_workspace_ints(int64_t n);
constexpr int kScanItemsU8 = 16;                      // flags per thread of the u8 compaction
constexpr int kScanTileBytes = kBlock * kScanItemsU8;  // flags per tile (4096)
// Hook of voxel_down_sample_hooked: called with the kept table's geometry
// (geom[8] = -1: occupancy unknown yet) and the table, after the voxel
// kernels are queued and before the representative count is read back.
typedef int (*VoxelHook)(void* ctx, const double* geom12, const void* vox);
int voxel_down_sample_hooked(const float* xyz, int64_t n, const double* min_bound, const double* max_bound,
                             double voxel_size, int32_t* rep_idx, float* rep_xyz, int64_t* m_host, float* voxel_pts,
                             int64_t voxel_cells, double* geom, void* ws, size_t ws_bytes, void* stream,
                             VoxelHook hook, void* ctx);
int compact_flags_scan(const uint8_t* flags, int64_t n, int64_t* count_dev, int32_t* tmp, hipStream_t s);
int compact_flags(const uint8_t* flags, int64_t n, int32_t* idx_out, int32_t* pos_out,
                  int64_t* count_dev, int32_t* tmp, hipStream_t s);

// Column reduction of a row-major partials matrix part[rows][width] -> out[width]
// with a fixed summation order (deterministic).  One block per 64 columns.
enum class RedOp { kSumF64, kSumI64, kMinF32, kMaxF32 };
int reduce_columns_f64(const double* part, int64_t rows, int width, double* out, hipStream_t s);
int reduce_columns_i32_to_i64(const int32_t* part, int64_t rows, int width, int64_t* out, hipStream_t s);

// AABB on device into a device double[6] (no sync).
size_t aabb_ws_bytes(int64_t n);
int aabb_device(const float* xyz, int64_t n, double* mm_dev, void* ws, hipStream_t s);

}  // namespace o3dx
