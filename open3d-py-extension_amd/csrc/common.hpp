// common.hpp — shared host/device helpers of libo3dx (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
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

// ------------------------------------------- exact (order-free) float sums
// "fx" sums: a float64 term t with |t| <= B becomes the integer
// v = round(t * 2^-q), q = fx_exp(B) = (frexp exponent of B) - kFxBits, so
// |v| < 2^51, and the integers are summed.  Integer addition is associative:
// a sum is the same bits for any lane, block or rank split — what the
// multi-GPU path needs (results identical for 1/2/4/8 GPUs)
// and what a float64 reduction cannot give.  One fma does the conversion:
// fma(t, 2^-q, 1.5 * 2^52) rounds t * 2^-q (exact: a power-of-two scale) to
// the nearest integer, whose bits minus the magic's bits are v.  A lane adds
// up to kFxLaneTerms terms in one int64 (< 2^63); across lanes, blocks and
// ranks the sums travel as two int64 digits {lo = low 32 bits (>= 0), hi =
// the rest}, which cannot overflow for < 2^31 terms.  The value is rounded to
// float64 once, at the end (fx_to_double).  Error: <= n 2^-52 B (round to
// nearest per term), the same order as a float64 sum's, but order-free.
constexpr int kFxBits = 51;
constexpr int64_t kFxLaneTerms = 4096;
constexpr double kFxMagic = 6755399441055744.0;  // 1.5 * 2^52
constexpr int64_t kFxMagicBits = 0x4338000000000000ll;

inline int fx_exp(double B) {
  int e = 0;
  const double b = (B > 0.0 && std::isfinite(B)) ? std::max(B, std::ldexp(1.0, -900)) : 1.0;
  std::frexp(b, &e);
  return e - kFxBits;
}
inline double fx_scale(int q) { return std::ldexp(1.0, -q); }

__device__ __forceinline__ int64_t fx_term(double t, double scale) {
  return (int64_t)__double_as_longlong(fma(t, scale, kFxMagic)) - kFxMagicBits;
}

// Block partial of K lane accumulators: out[2k] = sum of the low 32-bit
// digits, out[2k+1] = sum of the high parts (valid after the call in every
// thread's view of `out`, written by threads < 2K).  sh: (BLOCK/64) * 2K.
template <int BLOCK, int K>
__device__ __forceinline__ void block_fx(const int64_t (&acc)[K], int64_t* sh, int64_t* out) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    int64_t lo = acc[k] & 0xffffffffll, hi = acc[k] >> 32;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo += __shfl_xor(lo, o, 64);
      hi += __shfl_xor(hi, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      sh[w * 2 * K + 2 * k] = lo;
      sh[w * 2 * K + 2 * k + 1] = hi;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * K; t += BLOCK) {
    int64_t s = 0;
#pragma unroll
    for (int v = 0; v < BLOCK / 64; ++v) s += sh[v * 2 * K + t];
    out[t] = s;
  }
  __syncthreads();
}

// The exact value of a {lo, hi} digit sum (lo >= 0) scaled by 2^q, correctly
// rounded once: the carry of lo moves into hi (|hi| < 2^53), then
// hi 2^32 + lo is one rounded addition of two exact doubles — the same value
// as core.hip's fx_to_double (__int128), on the host and on the device.
__host__ __device__ inline double fx_value(int64_t lo, int64_t hi, int q) {
  const int64_t h = hi + (lo >> 32);
  const int64_t l = lo & 0xffffffffll;
  return ldexp(ldexp((double)h, 32) + (double)l, q);
}

// {lo, hi} digit sums + exponent of k sums (row j: {lo, hi, q, 0}) -> float64,
// correctly rounded (one rounding of the exact integer, then the exact scale)
void fx_to_double(const int64_t* fx4, int64_t k, double* out);
// digit sums (k rows {lo, hi}) + per-sum exponents -> the ABI's {lo, hi, q, 0} rows
inline void fx_pack(const int64_t* digits, const int* q, int64_t k, int64_t* fx4) {
  for (int64_t j = 0; j < k; ++j) {
    fx4[4 * j] = digits[2 * j];
    fx4[4 * j + 1] = digits[2 * j + 1];
    fx4[4 * j + 2] = q[j];
    fx4[4 * j + 3] = 0;
  }
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
// a device byte range to clear (folded into a kernel that runs anyway)
struct ZeroSpan {
  uint8_t* p = nullptr;
  size_t bytes = 0;
};
// Hook of voxel_down_sample_hooked: called with the kept table's geometry
// (geom[8] = -1: occupancy unknown yet) and the table, after the voxel
// kernels are queued and before the representative count is read back.
typedef int (*VoxelHook)(void* ctx, const double* geom12, const void* vox);
int voxel_down_sample_hooked(const float* xyz, int64_t n, const double* min_bound, const double* max_bound,
                             double voxel_size, int32_t* rep_idx, float* rep_xyz, int64_t* m_host, float* voxel_pts,
                             int64_t voxel_cells, double* geom, void* ws, size_t ws_bytes, void* stream,
                             VoxelHook hook, void* ctx, ZeroSpan extra_zero = {});
// A few words straight to the host: one kernel thread stores them into mapped
// pinned memory followed by a sequence number the host polls (no copy kernel
// in the stream, no event).  post_prepare takes the next sequence number of
// this host thread's post box; post_wait polls it (falling back to a stream
// wait) and copies the words out.
struct HostPost {
  uint64_t* words = nullptr;  // device view of the mapped words (<= kPostWords)
  volatile uint64_t* seq_word = nullptr;
  uint64_t seq = 0;
};
constexpr int kPostWords = 8;
int post_prepare(HostPost* p);
int post_wait(const HostPost& p, void* dst, size_t bytes, hipStream_t s);
__device__ __forceinline__ void post_publish(const HostPost& p, const int64_t* src, int nwords) {
  for (int i = 0; i < nwords; ++i) p.words[i] = (uint64_t)src[i];
  __threadfence_system();
  *p.seq_word = p.seq;
}

int compact_flags_scan(const uint8_t* flags, int64_t n, int64_t* count_dev, int32_t* tmp, hipStream_t s);
// post (nullable): count_dev[0 .. post_words) is published to the host once
// the total is known (the earlier words were final before the compaction)
int compact_flags(const uint8_t* flags, int64_t n, int32_t* idx_out, int32_t* pos_out,
                  int64_t* count_dev, int32_t* tmp, hipStream_t s, const HostPost* post = nullptr,
                  int post_words = 0);

// --------------------------------------------------------------- bounds
// zero [p, p + bytes) with the whole grid (16-B stores on the aligned middle)
__device__ __forceinline__ void grid_zero(uint8_t* p, size_t bytes) {
  if (!p || !bytes) return;
  const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  const size_t head = std::min(bytes, (size_t)((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15));
  const size_t nv = (bytes - head) / 16;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  for (size_t k = t0; k < nv; k += st) q[k] = make_uint4(0, 0, 0, 0);
  for (size_t k = t0; k < head; k += st) p[k] = 0;
  for (size_t k = head + nv * 16 + t0; k < bytes; k += st) p[k] = 0;
}

// This thread's share of a grid-strided min / max over an (n,3) float32
// cloud.  Aligned clouds are read as 16-B vectors, four points per three
// loads (x y z x | y z x y | z x y z), two chunks in flight per lane; the rows
// past the last whole chunk (and unaligned clouds) one point at a time.
__device__ __forceinline__ void aabb_accumulate(const float* __restrict__ xyz, int64_t n, float mn[3], float mx[3]) {
  for (int a = 0; a < 3; ++a) {
    mn[a] = INFINITY;
    mx[a] = -INFINITY;
  }
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  int64_t i0 = 0;
  if ((reinterpret_cast<uintptr_t>(xyz) & 15) == 0) {
    const float4* q = reinterpret_cast<const float4*>(xyz);
    const int64_t nch = n / 4;
    i0 = nch * 4;
    auto take = [&](const float4 a, const float4 b, const float4 d) {
      mn[0] = fminf(mn[0], fminf(fminf(a.x, a.w), fminf(b.z, d.y)));
      mn[1] = fminf(mn[1], fminf(fminf(a.y, b.x), fminf(b.w, d.z)));
      mn[2] = fminf(mn[2], fminf(fminf(a.z, b.y), fminf(d.x, d.w)));
      mx[0] = fmaxf(mx[0], fmaxf(fmaxf(a.x, a.w), fmaxf(b.z, d.y)));
      mx[1] = fmaxf(mx[1], fmaxf(fmaxf(a.y, b.x), fmaxf(b.w, d.z)));
      mx[2] = fmaxf(mx[2], fmaxf(fmaxf(a.z, b.y), fmaxf(d.x, d.w)));
    };
    int64_t c = t0;
    for (; c + st < nch; c += 2 * st) {
      const float4 a = q[3 * c], b = q[3 * c + 1], d = q[3 * c + 2];
      const float4 a2 = q[3 * (c + st)], b2 = q[3 * (c + st) + 1], d2 = q[3 * (c + st) + 2];
      take(a, b, d);
      take(a2, b2, d2);
    }
    if (c < nch) take(q[3 * c], q[3 * c + 1], q[3 * c + 2]);
  }
  for (int64_t i = i0 + t0; i < n; i += st) {
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    mn[0] = fminf(mn[0], x);
    mn[1] = fminf(mn[1], y);
    mn[2] = fminf(mn[2], z);
    mx[0] = fmaxf(mx[0], x);
    mx[1] = fmaxf(mx[1], y);
    mx[2] = fmaxf(mx[2], z);
  }
}

// min / max of the block's threads (6 columns: min x y z, max x y z) into
// out6 (written by threads 0..5); sh: kBlock / 64 x 6 floats of LDS
__device__ __forceinline__ void aabb_block_fold(float mn[3], float mx[3], float (*sh)[6], float* out6) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
      mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
    }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int a = 0; a < 3; ++a) {
      sh[w][a] = mn[a];
      sh[w][3 + a] = mx[a];
    }
  __syncthreads();
  if (threadIdx.x < 6) {
    float r = sh[0][threadIdx.x];
    for (int k = 1; k < kBlock / 64; ++k)
      r = threadIdx.x < 3 ? fminf(r, sh[k][threadIdx.x]) : fmaxf(r, sh[k][threadIdx.x]);
    out6[threadIdx.x] = r;
  }
}

// Where the bounds' final kernel publishes {min, max}.
struct AabbOut {
  double* mm_host;              // mapped pinned memory (device view), then
  uint64_t seq;                 //   this sequence number into
  volatile uint64_t* seq_host;  //   the mailbox's word 0
};
struct AabbNoTail {
  __device__ void operator()(const double*) const {}
};

// The bounds' final fold (one block of kBlock threads) over the nb block
// partials of k_aabb_partial: publishes {min, max} to the host mailbox, then
// runs tail(mm) on thread 0 (the voxel path: the one-pass binning's plan, so
// no separate plan launch).
template <class Tail>
__global__ void __launch_bounds__(kBlock) k_aabb_final_tail(const float* __restrict__ part, int nb, int64_t n,
                                                            AabbOut o, Tail tail) {
  __shared__ float sh[kBlock / 64][6];
  __shared__ float fin[6];
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int b = threadIdx.x; b < nb; b += kBlock)
    for (int a = 0; a < 3; ++a) {
      mn[a] = fminf(mn[a], part[b * 6 + a]);
      mx[a] = fmaxf(mx[a], part[b * 6 + 3 + a]);
    }
  aabb_block_fold(mn, mx, sh, fin);
  __syncthreads();
  if (threadIdx.x == 0) {
    double mm[6];
    for (int a = 0; a < 6; ++a) mm[a] = n == 0 ? 0.0 : (double)fin[a];
    for (int a = 0; a < 6; ++a) o.mm_host[a] = mm[a];
    __threadfence_system();
    *o.seq_host = o.seq;
    tail(mm);
  }
}

// Queues the bounds' partial kernel (z0..z3: clears folded in) and returns the
// mailbox of this host thread for the final kernel (advancing the sequence
// number aabb_end waits for); *part, *nb: the partials the final kernel folds.
int aabb_begin_partial(const float* xyz, int64_t n, void* ws, hipStream_t s, ZeroSpan z0, ZeroSpan z1, ZeroSpan z2,
                       ZeroSpan z3, AabbOut* o, const float** part, int* nb);

// Column reduction of a row-major partials matrix part[rows][width] -> out[width]
// with a fixed summation order (deterministic).  One block per 64 columns.
enum class RedOp { kSumF64, kSumI64, kMinF32, kMaxF32 };
int reduce_columns_f64(const double* part, int64_t rows, int width, double* out, hipStream_t s);
int reduce_columns_i32_to_i64(const int32_t* part, int64_t rows, int width, int64_t* out, hipStream_t s);
// int64 columns (fx digit partials): exact, any order
int reduce_columns_i64(const int64_t* part, int64_t rows, int width, int64_t* out, hipStream_t s);

// AABB on device into a device double[6] (no sync).
size_t aabb_ws_bytes(int64_t n);
int aabb_device(const float* xyz, int64_t n, double* mm_dev, void* ws, hipStream_t s);
// The bounds straight to the host: the final kernel writes them into mapped
// pinned memory followed by a sequence number the host polls (no copy kernel,
// no stream query).  aabb_begin queues the kernels (work queued after it
// keeps running while the host waits); aabb_end waits and returns {min, max}.
// z0..z3: device ranges the AABB kernel zeroes on the way (clears folded in;
// ZeroSpan above)
int aabb_begin(const float* xyz, int64_t n, void* ws, hipStream_t s, ZeroSpan z0 = {}, ZeroSpan z1 = {},
               ZeroSpan z2 = {}, ZeroSpan z3 = {});
int aabb_end(double mm_host[6], hipStream_t s);
// AABB of float64 points into a device double[6] (no sync); ws: aabb64_ws_bytes
size_t aabb64_ws_bytes();
int aabb64_device(const double* xyz, int64_t n, double* mm_dev, void* ws, hipStream_t s);

}  // namespace o3dx
