// core.hip — error state, scans / flag compaction, AABB reduction.
//
// AABB replaces o3d PointCloud.get_min_bound/get_max_bound
// (reference open3dpypro/PointCloud.py:145-146, :340).  HBM-bound: 12 B/point.
#include <cstdarg>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include <atomic>

#include "common.hpp"

namespace o3dx {

// ------------------------------------------------------------ kernel timing
static bool g_timing = false;
static std::mutex g_tmu;
struct Pending {
  std::string name;
  hipEvent_t a, b;
};
static std::vector<Pending> g_pending;
static std::map<std::string, std::pair<double, int64_t>> g_times;

static std::vector<hipEvent_t> g_free_events;  // recycled: no event creation on the launch path

bool timing_on() { return g_timing; }

// o3dx_kernel_timing_filter: when set, only the named timers record (the
// event records of the others stay out of a timed pipeline)
static std::string g_tfilter;
bool timing_wanted(const char* name) {
  if (!g_timing) return false;
  if (g_tfilter.empty()) return true;
  const std::string n = std::string(",") + name + ",";
  return (std::string(",") + g_tfilter + ",").find(n) != std::string::npos;
}

hipEvent_t timing_event() {
  {
    std::lock_guard<std::mutex> lk(g_tmu);
    if (!g_free_events.empty()) {
      hipEvent_t e = g_free_events.back();
      g_free_events.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

void timing_release(hipEvent_t e) {
  if (!e) return;
  std::lock_guard<std::mutex> lk(g_tmu);
  g_free_events.push_back(e);
}

int read_back(void* dst_host, const void* src_dev, size_t bytes, hipStream_t s) {
  // small read-backs go through a per-thread pinned staging buffer (a direct
  // DMA target; pageable destinations take the runtime's staged path)
  constexpr size_t kCap = 64 << 10;
  thread_local void* pin = nullptr;
  if (bytes <= kCap) {
    if (!pin && hipHostMalloc(&pin, kCap, hipHostMallocDefault) != hipSuccess) pin = nullptr;
    if (pin) {
      O3DX_HIP(hipMemcpyAsync(pin, src_dev, bytes, hipMemcpyDeviceToHost, s));
      O3DX_TRY(host_wait(s));
      std::memcpy(dst_host, pin, bytes);
      return 0;
    }
  }
  O3DX_HIP(hipMemcpyAsync(dst_host, src_dev, bytes, hipMemcpyDeviceToHost, s));
  return host_wait(s);
}

namespace {
struct PostBox {
  uint64_t* host = nullptr;  // [0] sequence, [1 ..] words (mapped, coherent)
  uint64_t* dev = nullptr;
  uint64_t seq = 0;
};
thread_local PostBox g_post;
}  // namespace

int post_prepare(HostPost* p) {
  PostBox& b = g_post;
  if (!b.host) {
    void* h = nullptr;
    O3DX_HIP(hipHostMalloc(&h, 256, hipHostMallocMapped | hipHostMallocCoherent));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return fail(O3DX_EIO, "post_prepare: no device view of the post box");
    }
    b.host = static_cast<uint64_t*>(h);
    b.dev = static_cast<uint64_t*>(d);
    b.host[0] = 0;
  }
  ++b.seq;
  p->words = b.dev + 1;
  p->seq_word = static_cast<volatile uint64_t*>(b.dev);
  p->seq = b.seq;
  return 0;
}

int post_wait(const HostPost& p, void* dst, size_t bytes, hipStream_t s) {
  if (bytes > kPostWords * sizeof(uint64_t)) return fail(O3DX_EINVAL, "post_wait: %zu bytes", bytes);
  volatile uint64_t* q = g_post.host;
  bool seen = false;
  for (int i = 0; i < (1 << 22) && !seen; ++i) seen = *q == p.seq;  // ~ms of polling
  if (!seen) {  // slow path: wait for the stream (errors surface here)
    O3DX_TRY(host_wait(s));
    seen = *q == p.seq;
    if (!seen) return fail(O3DX_EIO, "post_wait: the posted words never arrived");
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  std::memcpy(dst, const_cast<const uint64_t*>(g_post.host) + 1, bytes);
  return 0;
}

int host_wait(hipStream_t s) {
  // poll instead of a blocking wait: the short read-backs on the launch path
  // (counts, bounds) return as soon as the copy lands, without an interrupt
  // wake-up; falls back to the blocking wait after ~2 ms
  for (int i = 0; i < 4096; ++i) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) break;
  }
  O3DX_HIP(hipStreamSynchronize(s));
  return 0;
}

void timing_push(const char* name, hipEvent_t a, hipEvent_t b) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_pending.push_back({name, a, b});
}

static void timing_drain() {
  std::vector<Pending> p;
  {
    std::lock_guard<std::mutex> lk(g_tmu);
    p.swap(g_pending);
  }
  for (auto& e : p) {
    float ms = 0.f;
    if (hipEventSynchronize(e.b) == hipSuccess && hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
      std::lock_guard<std::mutex> lk(g_tmu);
      auto& t = g_times[e.name];
      t.first += ms;
      t.second += 1;
    }
    timing_release(e.a);
    timing_release(e.b);
  }
}

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// ------------------------------------------------------------------ scans
constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;  // 4096

__global__ void __launch_bounds__(kBlock) k_tile_sums_i32(const int32_t* __restrict__ in, int64_t n,
                                                          int32_t* __restrict__ part) {
  __shared__ int sh[kBlock / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = base + j;
    s += (i < n) ? in[i] : 0;
  }
  int tot;
  block_excl_scan<kBlock>(s, sh, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kBlock) k_tile_sums_u8(const uint8_t* __restrict__ f, int64_t n,
                                                         int32_t* __restrict__ part) {
  __shared__ int sh[kBlock / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int s = 0;
  if (base + kScanItems <= n) {
    uint4 v = *reinterpret_cast<const uint4*>(f + base);
    s = __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);  // flags are 0/1 bytes
  } else {
    for (int j = 0; j < kScanItems; ++j) {
      int64_t i = base + j;
      s += (i < n) ? (f[i] != 0) : 0;
    }
  }
  int tot;
  block_excl_scan<kBlock>(s, sh, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// Single-block exclusive scan of the tile partials (in place); total -> *total.
__global__ void __launch_bounds__(1024) k_scan_partials(int32_t* part, int64_t m, int32_t* total_i32,
                                                        int64_t* total_i64, HostPost post = {}, int post_words = 0) {
  __shared__ int sh[1024 / 64 + 1];
  int carry = 0;
  for (int64_t b = 0; b < m; b += 1024) {
    int64_t i = b + threadIdx.x;
    int v = (i < m) ? part[i] : 0;
    int tot;
    int ex = block_excl_scan<1024>(v, sh, &tot);
    if (i < m) part[i] = ex + carry;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    if (total_i32) *total_i32 = carry;
    if (total_i64) *total_i64 = carry;
    if (post.seq && total_i64) post_publish(post, total_i64, post_words);
  }
}

__global__ void __launch_bounds__(kBlock) k_tile_scan_i32(const int32_t* __restrict__ in, int64_t n,
                                                          const int32_t* __restrict__ part,
                                                          int32_t* __restrict__ out) {
  __shared__ int sh[kBlock / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int v[kScanItems];
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = base + j;
    v[j] = (i < n) ? in[i] : 0;
    s += v[j];
  }
  int tot;
  int ex = block_excl_scan<kBlock>(s, sh, &tot) + part[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = base + j;
    if (i < n) out[i] = ex;
    ex += v[j];
  }
}

__global__ void __launch_bounds__(kBlock) k_tile_compact_u8(const uint8_t* __restrict__ f, int64_t n,
                                                            const int32_t* __restrict__ part,
                                                            int32_t* __restrict__ idx_out,
                                                            int32_t* __restrict__ pos_out) {
  __shared__ int sh[kBlock / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  uint8_t v[kScanItems];
  if (base + kScanItems <= n) {
    uint4 q = *reinterpret_cast<const uint4*>(f + base);
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&q);
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) v[j] = b[j];
  } else {
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      int64_t i = base + j;
      v[j] = (i < n) ? f[i] : 0;
    }
  }
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) s += v[j] != 0;
  int tot;
  int ex = block_excl_scan<kBlock>(s, sh, &tot) + part[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = base + j;
    if (i < n) {
      if (pos_out) pos_out[i] = ex;
      if (v[j]) idx_out[ex++] = (int32_t)i;
    }
  }
}

// k_tile_compact_u8 with the tile's first output row formed in the block from
// the raw tile sums (no k_scan_partials launch: the block adds the sums of the
// tiles before it, at most a few thousand L2-resident words); the last tile
// writes the total.
__global__ void __launch_bounds__(kBlock) k_tile_compact_u8_sums(const uint8_t* __restrict__ f, int64_t n,
                                                                 const int32_t* __restrict__ part,
                                                                 int32_t* __restrict__ idx_out,
                                                                 int32_t* __restrict__ pos_out,
                                                                 int64_t* __restrict__ count_dev, HostPost post,
                                                                 int post_words) {
  __shared__ int sh[kBlock / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  uint8_t v[kScanItems];
  if (base + kScanItems <= n) {
    uint4 q = *reinterpret_cast<const uint4*>(f + base);
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&q);
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) v[j] = b[j];
  } else {
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      int64_t i = base + j;
      v[j] = (i < n) ? f[i] : 0;
    }
  }
  int p0 = 0;
  for (unsigned t = threadIdx.x; t < blockIdx.x; t += kBlock) p0 += part[t];
  int first;
  block_excl_scan<kBlock>(p0, sh, &first);
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) s += v[j] != 0;
  int tot;
  int ex = block_excl_scan<kBlock>(s, sh, &tot) + first;
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    *count_dev = (int64_t)first + tot;
    if (post.seq) post_publish(post, count_dev, post_words);
  }
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    int64_t i = base + j;
    if (i < n) {
      if (pos_out) pos_out[i] = ex;
      if (v[j]) idx_out[ex++] = (int32_t)i;
    }
  }
}

size_t scan_workspace_ints(int64_t n) { return (size_t)((n + kScanTile - 1) / kScanTile) + 64; }

int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* tmp, hipStream_t s) {
  int64_t tiles = (n + kScanTile - 1) / kScanTile;
  if (tiles == 0) {
    O3DX_HIP(hipMemsetAsync(out, 0, sizeof(int32_t), s));
    return 0;
  }
  hipLaunchKernelGGL(k_tile_sums_i32, dim3((unsigned)tiles), dim3(kBlock), 0, s, in, n, tmp);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, s, tmp, tiles, out + n, (int64_t*)nullptr);
  hipLaunchKernelGGL(k_tile_scan_i32, dim3((unsigned)tiles), dim3(kBlock), 0, s, in, n, tmp, out);
  O3DX_HIP(hipGetLastError());
  return 0;
}

size_t compact_workspace_ints(int64_t n) { return scan_workspace_ints(n); }

// The tile partial sums of compact_flags, scanned (tmp[tile] = the tile's
// first output row; *count_dev = total): for callers with their own
// compaction kernel over the same tiles (kScanTileBytes flags per tile).
int compact_flags_scan(const uint8_t* flags, int64_t n, int64_t* count_dev, int32_t* tmp, hipStream_t s) {
  int64_t tiles = (n + kScanTile - 1) / kScanTile;
  if (tiles == 0) {
    O3DX_HIP(hipMemsetAsync(count_dev, 0, sizeof(int64_t), s));
    return 0;
  }
  hipLaunchKernelGGL(k_tile_sums_u8, dim3((unsigned)tiles), dim3(kBlock), 0, s, flags, n, tmp);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, s, tmp, tiles, (int32_t*)nullptr, count_dev);
  O3DX_HIP(hipGetLastError());
  return 0;
}

int compact_flags(const uint8_t* flags, int64_t n, int32_t* idx_out, int32_t* pos_out,
                  int64_t* count_dev, int32_t* tmp, hipStream_t s, const HostPost* post, int post_words) {
  int64_t tiles = (n + kScanTile - 1) / kScanTile;
  const HostPost pp = post ? *post : HostPost{};
  if (post_words < 0 || post_words > kPostWords) return fail(O3DX_EINVAL, "compact_flags: %d post words", post_words);
  if (tiles == 0) {
    O3DX_HIP(hipMemsetAsync(count_dev, 0, sizeof(int64_t), s));
    if (post) return fail(O3DX_EINVAL, "compact_flags: nothing to post for an empty input");
    return 0;
  }
  hipLaunchKernelGGL(k_tile_sums_u8, dim3((unsigned)tiles), dim3(kBlock), 0, s, flags, n, tmp);
  if (tiles <= 4096) {  // the blocks read tiles^2 / 2 words in all (C2: 3M, from L2)
    hipLaunchKernelGGL(k_tile_compact_u8_sums, dim3((unsigned)tiles), dim3(kBlock), 0, s, flags, n, tmp, idx_out,
                       pos_out, count_dev, pp, post_words);
  } else {
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, s, tmp, tiles, (int32_t*)nullptr, count_dev, pp,
                       post_words);
    hipLaunchKernelGGL(k_tile_compact_u8, dim3((unsigned)tiles), dim3(kBlock), 0, s, flags, n, tmp, idx_out,
                       pos_out);
  }
  O3DX_HIP(hipGetLastError());
  return 0;
}

// -------------------------------------------------------- column reductions
// block = 64 columns x 16 row-groups; each thread sums its row-group's rows in
// order, then the 16 group partials are added in group order.
template <class T, class R>
__global__ void __launch_bounds__(1024) k_reduce_columns(const T* __restrict__ part, int64_t rows, int width,
                                                         R* __restrict__ out) {
  __shared__ R sh[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  R acc = 0;
  if (c < width)
    for (int64_t r = g; r < rows; r += 16) acc += (R)part[r * width + c];
  sh[g][threadIdx.x & 63] = acc;
  __syncthreads();
  if (g == 0 && c < width) {
    R t = 0;
    for (int k = 0; k < 16; ++k) t += sh[k][threadIdx.x & 63];
    out[c] = t;
  }
}

int reduce_columns_f64(const double* part, int64_t rows, int width, double* out, hipStream_t s) {
  hipLaunchKernelGGL((k_reduce_columns<double, double>), dim3((width + 63) / 64), dim3(1024), 0, s, part, rows, width,
                     out);
  O3DX_HIP(hipGetLastError());
  return 0;
}

// Integer columns: the rows are split over blockIdx.y as well (a few columns
// x thousands of rows would leave one block per 64 columns streaming every
// row), each block adding its partial column sums with a 64-bit integer
// atomic — integer addition, so the result is the same in any order.
constexpr int64_t kRedRowsPerBlock = 128;

template <class T>
__global__ void __launch_bounds__(1024) k_reduce_columns_i64(const T* __restrict__ part, int64_t rows, int width,
                                                             int64_t* __restrict__ out) {
  __shared__ int64_t sh[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * kRedRowsPerBlock, r1 = min(rows, r0 + kRedRowsPerBlock);
  int64_t acc = 0;
  if (c < width)
    for (int64_t r = r0 + g; r < r1; r += 16) acc += (int64_t)part[r * width + c];
  sh[g][threadIdx.x & 63] = acc;
  __syncthreads();
  if (g == 0 && c < width) {
    int64_t t = 0;
    for (int k = 0; k < 16; ++k) t += sh[k][threadIdx.x & 63];
    if (t) atomicAdd(reinterpret_cast<unsigned long long*>(&out[c]), (unsigned long long)t);
  }
}

template <class T>
static int reduce_columns_to_i64(const T* part, int64_t rows, int width, int64_t* out, hipStream_t s) {
  if (width <= 0) return 0;
  O3DX_HIP(hipMemsetAsync(out, 0, (size_t)width * sizeof(int64_t), s));
  const int64_t by = std::max<int64_t>(1, (rows + kRedRowsPerBlock - 1) / kRedRowsPerBlock);
  if (by > 65535) return fail(O3DX_EINVAL, "reduce_columns: too many rows");
  hipLaunchKernelGGL(k_reduce_columns_i64<T>, dim3((width + 63) / 64, (unsigned)by), dim3(1024), 0, s, part, rows,
                     width, out);
  O3DX_HIP(hipGetLastError());
  return 0;
}

int reduce_columns_i32_to_i64(const int32_t* part, int64_t rows, int width, int64_t* out, hipStream_t s) {
  return reduce_columns_to_i64(part, rows, width, out, s);
}

int reduce_columns_i64(const int64_t* part, int64_t rows, int width, int64_t* out, hipStream_t s) {
  return reduce_columns_to_i64(part, rows, width, out, s);
}

void fx_to_double(const int64_t* fx4, int64_t k, double* out) {
  for (int64_t j = 0; j < k; ++j) {
    const __int128 v = (__int128)fx4[4 * j + 1] * ((__int128)1 << 32) + (__int128)fx4[4 * j];
    out[j] = std::ldexp((double)v, (int)fx4[4 * j + 2]);  // (double) of __int128: round to nearest even
  }
}

// ------------------------------------------------------------------- AABB
constexpr int kAabbBlocks = 1024;

// per-block partial {min, max} (the two-launch form: aabb_device)
__global__ void __launch_bounds__(kBlock) k_aabb_partial(const float* __restrict__ xyz, int64_t n,
                                                         float* __restrict__ part, ZeroSpan z0 = {},
                                                         ZeroSpan z1 = {}, ZeroSpan z2 = {}, ZeroSpan z3 = {}) {
  grid_zero(z0.p, z0.bytes);
  grid_zero(z1.p, z1.bytes);
  grid_zero(z2.p, z2.bytes);
  grid_zero(z3.p, z3.bytes);
  float mn[3], mx[3];
  aabb_accumulate(xyz, n, mn, mx);
  __shared__ float sh[kBlock / 64][6];
  aabb_block_fold(mn, mx, sh, part + (size_t)blockIdx.x * 6);
}

__global__ void __launch_bounds__(1024) k_aabb_final(const float* __restrict__ part, int nb, int64_t n,
                                                     double* __restrict__ mm) {
  // 6 columns x 170 row-groups; min/max are order-independent
  __shared__ float sh[6][171];
  const int a = threadIdx.x % 6, g = threadIdx.x / 6;
  if (g < 170) {
    float r = a < 3 ? INFINITY : -INFINITY;
    for (int b = g; b < nb; b += 170) r = a < 3 ? fminf(r, part[b * 6 + a]) : fmaxf(r, part[b * 6 + a]);
    sh[a][g] = r;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    float r = sh[a][0];
    for (int k = 1; k < 170; ++k) r = a < 3 ? fminf(r, sh[a][k]) : fmaxf(r, sh[a][k]);
    mm[a] = n == 0 ? 0.0 : (double)r;
  }
}

namespace {
struct AabbMailbox {
  uint64_t* host = nullptr;  // [0] sequence, [1..6] bounds (mapped, coherent)
  uint64_t* dev = nullptr;
  uint64_t seq = 0;
};
thread_local AabbMailbox g_ambox;
}  // namespace

int aabb_begin_partial(const float* xyz, int64_t n, void* ws, hipStream_t s, ZeroSpan z0, ZeroSpan z1, ZeroSpan z2,
                       ZeroSpan z3, AabbOut* o, const float** part, int* nb) {
  AabbMailbox& m = g_ambox;
  if (!m.host) {
    void* h = nullptr;
    O3DX_HIP(hipHostMalloc(&h, 256, hipHostMallocMapped | hipHostMallocCoherent));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return fail(O3DX_EIO, "aabb_begin: no device view of the mailbox");
    }
    m.host = static_cast<uint64_t*>(h);
    m.dev = static_cast<uint64_t*>(d);
    m.host[0] = 0;
  }
  ++m.seq;
  o->mm_host = reinterpret_cast<double*>(m.dev + 1);
  o->seq = m.seq;
  o->seq_host = static_cast<volatile uint64_t*>(m.dev);
  float* pt = reinterpret_cast<float*>(ws);
  int b = (int)std::min<int64_t>(kAabbBlocks, std::max<int64_t>(1, (n + kBlock - 1) / kBlock));
  if (z0.bytes || z1.bytes || z2.bytes || z3.bytes) b = kAabbBlocks;  // the clears want the whole grid
  hipLaunchKernelGGL(k_aabb_partial, dim3(b), dim3(kBlock), 0, s, xyz, n, pt, z0, z1, z2, z3);
  *part = pt;
  *nb = b;
  return 0;
}

int aabb_begin(const float* xyz, int64_t n, void* ws, hipStream_t s, ZeroSpan z0, ZeroSpan z1, ZeroSpan z2,
               ZeroSpan z3) {
  AabbOut o;
  const float* part;
  int nb;
  O3DX_TRY(aabb_begin_partial(xyz, n, ws, s, z0, z1, z2, z3, &o, &part, &nb));
  hipLaunchKernelGGL(k_aabb_final_tail<AabbNoTail>, dim3(1), dim3(kBlock), 0, s, part, nb, n, o, AabbNoTail{});
  O3DX_HIP(hipGetLastError());
  return 0;
}

int aabb_end(double mm_host[6], hipStream_t s) {
  AabbMailbox& m = g_ambox;
  volatile uint64_t* q = m.host;
  bool seen = false;
  for (int i = 0; i < (1 << 22) && !seen; ++i) seen = *q == m.seq;  // ~ms of polling
  if (!seen) {  // slow path: wait for the stream (errors surface here)
    O3DX_TRY(host_wait(s));
    seen = *q == m.seq;
    if (!seen) return fail(O3DX_EIO, "aabb_end: bounds never arrived");
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  std::memcpy(mm_host, const_cast<const uint64_t*>(m.host) + 1, 6 * sizeof(double));
  return 0;
}

size_t aabb_ws_bytes(int64_t) { return Arena::align(kAabbBlocks * 6 * sizeof(float)) + 256; }

int aabb_device(const float* xyz, int64_t n, double* mm_dev, void* ws, hipStream_t s) {
  float* part = reinterpret_cast<float*>(ws);
  int nb = (int)std::min<int64_t>(kAabbBlocks, std::max<int64_t>(1, (n + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_aabb_partial, dim3(nb), dim3(kBlock), 0, s, xyz, n, part);
  hipLaunchKernelGGL(k_aabb_final, dim3(1), dim3(1024), 0, s, part, nb, n, mm_dev);
  O3DX_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------- float64 AABB
// The float64 boundary (o3dx_*_f64): min / max per axis of an (n,3) float64
// cloud, Geometry3D::ComputeMinBound/MaxBound on Open3D's float64 storage.
// Block partials then one final block (min / max are order-independent).
constexpr int kAabb64Blocks = 1024;

__global__ void __launch_bounds__(kBlock) k_aabb64_partial(const double* __restrict__ xyz, int64_t n,
                                                           double* __restrict__ part) {
  double mn[3] = {INFINITY, INFINITY, INFINITY};
  double mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const double v = xyz[3 * i + a];
      mn[a] = fmin(mn[a], v);
      mx[a] = fmax(mx[a], v);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      mn[a] = fmin(mn[a], __shfl_xor(mn[a], o, 64));
      mx[a] = fmax(mx[a], __shfl_xor(mx[a], o, 64));
    }
  __shared__ double sh[kBlock / 64][6];
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0)
    for (int a = 0; a < 3; ++a) {
      sh[w][a] = mn[a];
      sh[w][3 + a] = mx[a];
    }
  __syncthreads();
  if (threadIdx.x < 6) {
    double r = sh[0][threadIdx.x];
    for (int k = 1; k < kBlock / 64; ++k)
      r = threadIdx.x < 3 ? fmin(r, sh[k][threadIdx.x]) : fmax(r, sh[k][threadIdx.x]);
    part[blockIdx.x * 6 + threadIdx.x] = r;
  }
}

__global__ void __launch_bounds__(1024) k_aabb64_final(const double* __restrict__ part, int nb, int64_t n,
                                                       double* __restrict__ mm) {
  __shared__ double sh[6][171];
  const int a = threadIdx.x % 6, g = threadIdx.x / 6;
  if (g < 170) {
    double r = a < 3 ? INFINITY : -INFINITY;
    for (int b = g; b < nb; b += 170) r = a < 3 ? fmin(r, part[b * 6 + a]) : fmax(r, part[b * 6 + a]);
    sh[a][g] = r;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    double r = sh[a][0];
    for (int k = 1; k < 170; ++k) r = a < 3 ? fmin(r, sh[a][k]) : fmax(r, sh[a][k]);
    mm[a] = n == 0 ? 0.0 : r;
  }
}

size_t aabb64_ws_bytes() { return Arena::align(kAabb64Blocks * 6 * sizeof(double)) + 256; }

int aabb64_device(const double* xyz, int64_t n, double* mm_dev, void* ws, hipStream_t s) {
  double* part = reinterpret_cast<double*>(ws);
  const int nb = (int)std::min<int64_t>(kAabb64Blocks, std::max<int64_t>(1, (n + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_aabb64_partial, dim3(nb), dim3(kBlock), 0, s, xyz, n, part);
  hipLaunchKernelGGL(k_aabb64_final, dim3(1), dim3(1024), 0, s, part, nb, n, mm_dev);
  O3DX_HIP(hipGetLastError());
  return 0;
}

}  // namespace o3dx

using namespace o3dx;

extern "C" size_t o3dx_aabb_f64_workspace_bytes(int64_t) { return aabb64_ws_bytes() + 256; }

extern "C" int o3dx_aabb_f64(const double* xyz, int64_t n, double* minmax_host, void* ws, size_t ws_bytes,
                             void* stream) {
  if (n < 0 || (n > 0 && !xyz) || !minmax_host) return fail(O3DX_EINVAL, "o3dx_aabb_f64: bad arguments");
  if (!ws || ws_bytes < o3dx_aabb_f64_workspace_bytes(n)) return fail(O3DX_ENOMEM, "o3dx_aabb_f64: workspace too small");
  hipStream_t s = as_stream(stream);
  double* mm = reinterpret_cast<double*>((char*)ws + aabb64_ws_bytes());
  O3DX_TRY(aabb64_device(xyz, n, mm, ws, s));
  O3DX_TRY(read_back(minmax_host, mm, 6 * sizeof(double), s));
  return 0;
}

extern "C" int o3dx_abi_version(void) { return O3DX_ABI_VERSION; }

extern "C" void o3dx_set_kernel_timing(int enable) {
  if (!enable) timing_drain();
  g_timing = enable != 0;
}

extern "C" void o3dx_kernel_timing_filter(const char* names_csv) { g_tfilter = names_csv ? names_csv : ""; }

extern "C" void o3dx_reset_kernel_timing(void) {
  timing_drain();
  std::lock_guard<std::mutex> lk(g_tmu);
  g_times.clear();
}

extern "C" int o3dx_kernel_timing(const char* name, double* total_ms, int64_t* launches) {
  timing_drain();
  std::lock_guard<std::mutex> lk(g_tmu);
  auto it = g_times.find(name ? name : "");
  if (it == g_times.end()) {
    if (total_ms) *total_ms = 0;
    if (launches) *launches = 0;
    return -1;
  }
  if (total_ms) *total_ms = it->second.first;
  if (launches) *launches = it->second.second;
  return 0;
}

extern "C" const char* o3dx_last_error(void) { return g_err.c_str(); }

extern "C" int o3dx_fx_to_double(const int64_t* fx4, int64_t k, double* out) {
  if (k < 0 || (k > 0 && (!fx4 || !out))) return fail(O3DX_EINVAL, "o3dx_fx_to_double: bad arguments");
  fx_to_double(fx4, k, out);
  return 0;
}

extern "C" size_t o3dx_aabb_workspace_bytes(int64_t n) { return aabb_ws_bytes(n) + 256; }

extern "C" int o3dx_aabb_device(const float* xyz, int64_t n, double* minmax_dev, void* ws, size_t ws_bytes,
                                void* stream) {
  if (n < 0 || (n > 0 && !xyz) || !minmax_dev) return fail(O3DX_EINVAL, "o3dx_aabb_device: bad arguments");
  if (!ws || ws_bytes < o3dx_aabb_workspace_bytes(n)) return fail(O3DX_ENOMEM, "o3dx_aabb_device: workspace too small");
  return aabb_device(xyz, n, minmax_dev, ws, as_stream(stream));
}

extern "C" int o3dx_aabb(const float* xyz, int64_t n, double* minmax_host, void* ws, size_t ws_bytes,
                         void* stream) {
  if (n < 0 || (n > 0 && !xyz) || !minmax_host) return fail(O3DX_EINVAL, "o3dx_aabb: bad arguments");
  if (!ws || ws_bytes < o3dx_aabb_workspace_bytes(n))
    return fail(O3DX_ENOMEM, "o3dx_aabb: workspace too small");
  hipStream_t s = as_stream(stream);
  char* w = (char*)ws;
  double* mm = reinterpret_cast<double*>(w + aabb_ws_bytes(n));
  O3DX_TRY(aabb_device(xyz, n, mm, w, s));
  O3DX_TRY(read_back(minmax_host, mm, 6 * sizeof(double), s));
  return 0;
}
