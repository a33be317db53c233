// ransac.hip — segment_plane (RANSAC) with Open3D semantics.
//
// Replaces o3d PointCloud.segment_plane(distance_threshold, ransac_n,
// num_iterations, probability) (reference open3dpypro/PointCloud.py:75-77,
// processors.py:637-638 PlaneDetection.cpu_model, seg_planes :941-985).
// Restated from Open3D geometry/PointCloudSegmentation.cpp (SegmentPlane,
// EvaluateRANSACBasedOnDistance, GetPlaneFromPoints, RandomSampler) and
// TriangleMesh::ComputeTrianglePlane.
//
// GPU design: every hypothesis is scored against every point in ONE sweep
// (hypotheses are independent; Open3D's sequential selection with early break
// is replayed on the host afterwards, which cannot change any score).  Each
// lane holds 4 points in registers; plane coefficients are wave-uniform
// (scalar loads); a float32 FMA distance with a per-hypothesis error band
// decides almost every point, lanes inside the band are re-decided in float64
// exactly as Open3D evaluates |(a x + c z) + (b y + d)| < thr; inlier counts
// are ballot-popcounts into LDS.  Sigma|d| (only needed to break fitness ties)
// is computed exactly in float64 for the tied hypotheses only.
#include <cstring>
#include <random>
#include <vector>

#include "common.hpp"
#include "grid.hpp"

namespace o3dx {

constexpr int kPts = 16;
constexpr int kHChunk = 1024;
constexpr int kCountBlocksMax = 4096;

struct P3 {
  float x, y, z;
};

__device__ __forceinline__ double plane_dist64(const double* pl, double x, double y, double z) {
  // Eigen Vector4d dot packet order: (a*x + c*z) + (b*y + d*1)
  double ax = pl[0] * x, by = pl[1] * y, cz = pl[2] * z, dw = pl[3] * 1.0;
  return fabs((ax + cz) + (by + dw));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// One block sweeps tiles of kBlock * kPts points against hypotheses
// [h0, h0 + hc).  Points past n are NaN (every comparison false, no masks).
// The next hypothesis' coefficients are loaded while the current one is
// evaluated; distances of two points per packed FMA.
__global__ void __launch_bounds__(kBlock) k_plane_count(const float* __restrict__ xyz, int64_t n,
                                                        const float4* __restrict__ pl32,
                                                        const float4* __restrict__ band,
                                                        const double* __restrict__ pl64, int H, int h0, int hc,
                                                        double thr, int32_t* __restrict__ partial) {
  static_assert(kPts % 2 == 0, "points are processed in pairs");
  constexpr int kPairs = kPts / 2;
  __shared__ int cnt[kHChunk];
  for (int h = threadIdx.x; h < hc; h += kBlock) cnt[h] = 0;
  __syncthreads();
  const P3* p = reinterpret_cast<const P3*>(xyz);
  const int64_t tile = (int64_t)kBlock * kPts;
  const float qnan = __int_as_float(0x7fc00000);
  for (int64_t base = (int64_t)blockIdx.x * tile; base < n; base += (int64_t)gridDim.x * tile) {
    f32x2 X[kPairs], Y[kPairs], Z[kPairs];
#pragma unroll
    for (int k = 0; k < kPairs; ++k) {
      const int64_t i0 = base + (int64_t)(2 * k) * kBlock + threadIdx.x, i1 = i0 + kBlock;
      const P3 a = i0 < n ? p[i0] : P3{qnan, qnan, qnan};
      const P3 b = i1 < n ? p[i1] : P3{qnan, qnan, qnan};
      X[k] = (f32x2){a.x, b.x};
      Y[k] = (f32x2){a.y, b.y};
      Z[k] = (f32x2){a.z, b.z};
    }
    float4 P = pl32[h0];
    float4 B = band[h0];
    for (int h = 0; h < hc; ++h) {
      const int hn = (h + 1 < hc) ? h + 1 : h;
      const float4 Pn = pl32[h0 + hn];
      const float4 Bn = band[h0 + hn];
      int wc = 0;
      // ambiguity band [B.x, B.y) = mid B.z +- B.w (conservative): each lane
      // keeps its closest |e - mid| (VALU), one ballot per hypothesis
      float amb = INFINITY;
      // all distances first (independent chains), then the tests
      f32x2 D[kPairs];
#pragma unroll
      for (int k = 0; k < kPairs; ++k)
        D[k] = __builtin_elementwise_fma(
            (f32x2){P.x, P.x}, X[k],
            __builtin_elementwise_fma((f32x2){P.y, P.y}, Y[k],
                                      __builtin_elementwise_fma((f32x2){P.z, P.z}, Z[k], (f32x2){P.w, P.w})));
      __builtin_amdgcn_sched_barrier(0);
      float am[kPairs];
#pragma unroll
      for (int k = 0; k < kPairs; ++k) am[k] = fminf(fabsf(fabsf(D[k].x) - B.z), fabsf(fabsf(D[k].y) - B.z));
#pragma unroll
      for (int k = 0; k < kPairs; ++k)
        wc += __popcll(__ballot(fabsf(D[k].x) < B.x)) + __popcll(__ballot(fabsf(D[k].y) < B.x));
#pragma unroll
      for (int k = 0; k < kPairs; ++k) amb = fminf(amb, am[k]);
      if (__ballot(amb <= B.w)) {  // rare: re-decide band points in float64, Open3D's order
        const double* pl = pl64 + 4 * (h0 + h);
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
          const f32x2 d = __builtin_elementwise_fma(
              (f32x2){P.x, P.x}, X[k],
              __builtin_elementwise_fma((f32x2){P.y, P.y}, Y[k],
                                        __builtin_elementwise_fma((f32x2){P.z, P.z}, Z[k], (f32x2){P.w, P.w})));
          const float e0 = fabsf(d.x), e1 = fabsf(d.y);
          const bool x0 = !(e0 < B.x) && e0 < B.y && plane_dist64(pl, X[k].x, Y[k].x, Z[k].x) < thr;
          const bool x1 = !(e1 < B.x) && e1 < B.y && plane_dist64(pl, X[k].y, Y[k].y, Z[k].y) < thr;
          wc += __popcll(__ballot(x0)) + __popcll(__ballot(x1));
        }
      }
      if (lane_id() == 0 && wc) atomicAdd(&cnt[h], wc);
      P = Pn;
      B = Bn;
    }
  }
  __syncthreads();
  for (int h = threadIdx.x; h < hc; h += kBlock) partial[(int64_t)blockIdx.x * H + h0 + h] = cnt[h];
}

// ---------------------------------------------------------------------------
// The counts, one sweep over all hypotheses.  A wave holds a batch of 64 PL
// points (PL per lane, packed pairs) and HC hypotheses (planes read out of
// one register per coefficient with v_readlane: no memory latency in the
// loop).  One float32 window serves every hypothesis (the union of their
// windows [lo, hi)), tested on squares so that no |d| is needed:
//   d = fma(a, x, fma(b, y, fma(c, z, d)))   packed: 1.5 ops per point
//   t = fma(d, d, -Llo)                      packed: 0.5 (t < 0 <=> d^2 < Llo <= lo^2)
//   inliers: v_cmp t < 0, popcount on the scalar unit (counts are wave-uniform)
//   mn = umin(mn, bits(t))                   0 <= t <= fl(Lhi - Llo) covers lo <= |d| < hi
// Per batch and hypothesis one ballot of mn <= W marks window results; the
// wave stores one bit per hypothesis in the (batch, chunk) word of a bitmap,
// and k_plane_fixup re-decides those (batch, hypothesis) blocks in float64
// in Open3D's order.  Points past n are NaN: neither counted (t < 0 is
// false) nor in the window (their bits exceed W).  Blocks are mapped so that
// the waves sharing a batch range (all hypothesis chunks) run on one XCD
// (its L2 serves the re-reads of the points).
// Shapes: HC hypotheses per wave x PL points per lane per batch (batch =
// 64 PL points).  Default 32 x 16; O3DX_RANSAC_SHAPE=HCxPL picks another
// instantiated shape (tuning).
constexpr int kCountWaves = 2048;      // batch ranges (waves per hypothesis chunk)
constexpr int kMinBatchPts = 64 * 8;   // smallest instantiated batch (bitmap sizing)
constexpr int kMinHC = 16;             // smallest instantiated chunk (bitmap sizing)

template <int PL>
__device__ __forceinline__ void plane_batch_load(const P3* __restrict__ p, int64_t n, int64_t gb, int lane,
                                                 f32x2 (&X)[PL / 2], f32x2 (&Y)[PL / 2], f32x2 (&Z)[PL / 2]) {
  const float qnan = __int_as_float(0x7fc00000);
#pragma unroll
  for (int k = 0; k < PL / 2; ++k) {
    const int64_t i0 = gb * (64 * PL) + (int64_t)(2 * k) * 64 + lane, i1 = i0 + 64;
    // clamped, unconditional loads; rows past n become NaN afterwards
    const P3 a = p[min(i0, n - 1)];
    const P3 b = p[min(i1, n - 1)];
    X[k] = (f32x2){i0 < n ? a.x : qnan, i1 < n ? b.x : qnan};
    Y[k] = (f32x2){i0 < n ? a.y : qnan, i1 < n ? b.y : qnan};
    Z[k] = (f32x2){i0 < n ? a.z : qnan, i1 < n ? b.z : qnan};
  }
}

// two points' distances per packed fma (measured faster here than scalar
// fmas), each element the fmaf chain fma(a, x, fma(b, y, fma(c, z, d)))
__device__ __forceinline__ f32x2 plane_dist_pk(const float4 P, f32x2 x, f32x2 y, f32x2 z) {
  return __builtin_elementwise_fma((f32x2){P.x, P.x}, x,
                                   __builtin_elementwise_fma((f32x2){P.y, P.y}, y,
                                                             __builtin_elementwise_fma((f32x2){P.z, P.z}, z,
                                                                                       (f32x2){P.w, P.w})));
}

// t = d * d - L in one rounding: t < 0 <=> d^2 < L exactly (the sign of an
// fma is the sign of its exact value), so no |d| is needed and two points
// share one packed op
__device__ __forceinline__ f32x2 plane_sq_test(f32x2 d, float L) {
  return __builtin_elementwise_fma(d, d, (f32x2){-L, -L});
}

// block -> (batch range, group of 4 hypothesis chunks), XCD-aware: the
// launch's blocks are dealt round-robin over the 8 XCDs, so logical block
// l = (b % 8) * (nb / 8) + b / 8 puts consecutive l on one XCD.
__device__ __forceinline__ int xcd_logical_block(int b, int nb) {
  if (nb % 8) return b;
  return (b % 8) * (nb / 8) + b / 8;
}

template <int kHC, int kPL>  // kHC <= 32: one bitmap bit per hypothesis
__global__ void __launch_bounds__(kBlock) k_plane_count_v(const float* __restrict__ xyz, int64_t n,
                                                          const float4* __restrict__ pl32, int H, float Llo,
                                                          uint32_t wbits, int64_t batches_per_wave, int nwp,
                                                          int ncg, int32_t* __restrict__ partial,
                                                          uint32_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int wp = lb / ncg;                                                      // batch range
  const int chunk = __builtin_amdgcn_readfirstlane((lb % ncg) * (kBlock / 64) + (threadIdx.x >> 6));
  const int nchunks = (H + kHC - 1) / kHC;
  if (wp >= nwp || chunk >= nchunks) return;
  const int h0 = chunk * kHC;
  const P3* p = reinterpret_cast<const P3*>(xyz);
  int cnt = 0;  // lane h: hypothesis h0 + h's count (popcounts of its inlier ballots)
  // lane j holds plane h0 + (j % kHC) (h0 + j >= H: a copy of the last plane,
  // its counts never written back)
  float4 Pl = pl32[min(h0 + (lane % kHC), H - 1)];
  constexpr int kBatchPts = 64 * kPL;
  const int64_t nbatches = (n + kBatchPts - 1) / kBatchPts;
  for (int64_t b = 0; b < batches_per_wave; ++b) {
    const int64_t gb = (int64_t)wp * batches_per_wave + b;
    if (gb >= nbatches) break;
    // the planes are read out of Pl per batch, not hoisted out of the batch
    // loop into 128 scalar registers (an empty asm that "changes" Pl)
    asm volatile("" : "+v"(Pl.x), "+v"(Pl.y), "+v"(Pl.z), "+v"(Pl.w));
    f32x2 X[kPL / 2], Y[kPL / 2], Z[kPL / 2];
    plane_batch_load<kPL>(p, n, gb, lane, X, Y, Z);
    uint32_t word = 0;
#pragma unroll
    for (int h = 0; h < kHC; ++h) {
      // plane h from lane h (v_readlane into scalar registers: no memory
      // latency inside the loop)
      const float4 P = make_float4(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.x), h)),
                                   __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.y), h)),
                                   __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.z), h)),
                                   __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.w), h)));
      uint32_t mn = ~0u;
      int sc = 0;  // wave-uniform
#pragma unroll
      for (int k = 0; k < kPL / 2; ++k) {
        const f32x2 t = plane_sq_test(plane_dist_pk(P, X[k], Y[k], Z[k]), Llo);
        // inliers: one v_cmp per point, counted on the scalar unit
        sc += __popcll(__ballot(t.x < 0.0f)) + __popcll(__ballot(t.y < 0.0f));
        asm("" : "+s"(sc));  // summed as they come (a deferred sum tree spills the masks)
        mn = min(mn, min(__float_as_uint(t.x), __float_as_uint(t.y)));
      }
      cnt += lane == h ? sc : 0;
      if (__ballot(mn <= wbits)) word |= 1u << h;
    }
    if (lane == 0) flags[gb * nchunks + chunk] = word;
  }
  if (lane < kHC && h0 + lane < H) partial[(int64_t)wp * H + h0 + lane] = cnt;
}

// The window results of the flagged (batch, hypothesis) blocks decided in
// float64 (Open3D's order).  A wave per bitmap word: its batch's points are
// loaded once, then every flagged hypothesis is re-evaluated (the same packed
// fma chain: the same float32 distance), window results decided in float64,
// counted per lane, summed over the wave, one atomic per hypothesis.
template <int kHC, int kPL>
__global__ void __launch_bounds__(kBlock) k_plane_fixup(const float* __restrict__ xyz, int64_t n,
                                                        const float4* __restrict__ pl32,
                                                        const double* __restrict__ pl64, int H, double thr, float Llo,
                                                        uint32_t wbits, const uint32_t* __restrict__ flags,
                                                        int64_t nwords, int64_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int nchunks = (H + kHC - 1) / kHC;
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); w < nwords;
       w += (int64_t)gridDim.x * (kBlock / 64)) {
    uint32_t word = flags[w];
    if (!word) continue;
    const int64_t gb = w / nchunks;
    const int h0 = (int)(w % nchunks) * kHC;
    f32x2 X[kPL / 2], Y[kPL / 2], Z[kPL / 2];
    plane_batch_load<kPL>(p, n, gb, lane, X, Y, Z);
    while (word) {
      const int h = h0 + __ffs((int)word) - 1;
      word &= word - 1;
      if (h >= H) continue;
      const float4 P = pl32[h];
      const double* pl = pl64 + 4 * (int64_t)h;
      int c = 0;
#pragma unroll
      for (int k = 0; k < kPL / 2; ++k) {
        const f32x2 t = plane_sq_test(plane_dist_pk(P, X[k], Y[k], Z[k]), Llo);
        if (__float_as_uint(t.x) <= wbits && plane_dist64(pl, X[k].x, Y[k].x, Z[k].x) < thr) ++c;
        if (__float_as_uint(t.y) <= wbits && plane_dist64(pl, X[k].y, Y[k].y, Z[k].y) < thr) ++c;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
      if (lane == 0 && c) atomicAdd(reinterpret_cast<unsigned long long*>(&counts[h]), (unsigned long long)c);
    }
  }
}

// ---------------------------------------------------------------------------
// The counts over a cell grid of the cloud (grid.hpp: points grouped by
// cell, rows of cells along x contiguous).  Along a row the distance of the
// cell centres to a plane is affine in x, so the cells the slab
// |n.p + d| < thr can reach form one interval of x, found in float64 with a
// rigorous reach (|a|+|b|+|c|) (h/2 + assignment slack) and widened by a
// cell on each side; every other cell of the row holds no inlier.  The
// interval's points are one contiguous range of the sorted points.  A wave
// takes one hypothesis x 64 rows (a lane computes one row's range), cuts the
// ranges into chunks of 64 points and tests chunk after chunk with all
// lanes (coalesced loads, several chunks in flight), with the per-point
// window (t = fma(d, d, -Llo) < 0 certain, 0 <= t <= W decided in float64 in
// Open3D's order).
__global__ void __launch_bounds__(kBlock) k_plane_count_grid(GridView g, const float4* __restrict__ pl32,
                                                             const double* __restrict__ pl64, int H, double thr,
                                                             float Llo, uint32_t wbits, double cmargin,
                                                             int groups_per_h, int32_t* __restrict__ counts32) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t ntasks = (int64_t)H * groups_per_h;
  const int rows = g.ny * g.nz;
  for (int64_t t = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); t < ntasks; t += nwaves) {
    const int h = (int)(t / groups_per_h);
    const int row = (int)(t % groups_per_h) * 64 + lane;
    const float4 P = pl32[h];
    const double* pl = pl64 + 4 * (int64_t)h;
    const double a = pl[0], b = pl[1], c = pl[2], d = pl[3];
    int pa = 0, pb = 0;
    if (row < rows) {
      const int y = row % g.ny, z = row / g.ny;
      const double hh = (double)g.h;
      const double A = a * ((double)g.ox + 0.5 * hh) + b * ((double)g.oy + ((double)y + 0.5) * hh) +
                       c * ((double)g.oz + ((double)z + 0.5) * hh) + d;
      const double B = a * hh;
      const double T = thr + (fabs(a) + fabs(b) + fabs(c)) * (0.5 * hh + (double)g.slack) + cmargin;
      int x0 = 0, x1 = g.nx - 1;  // non-finite planes: the whole row (the points decide)
      if (isfinite(A) && isfinite(B)) {
        if (B != 0.0) {
          double u = (-T - A) / B, v = (T - A) / B;
          if (u > v) {
            const double w = u;
            u = v;
            v = w;
          }
          u = fmin(fmax(u, -2.0), (double)g.nx + 2.0);
          v = fmin(fmax(v, -2.0), (double)g.nx + 2.0);
          x0 = max((int)floor(u) - 1, 0);
          x1 = min((int)ceil(v) + 1, g.nx - 1);
        } else if (!(fabs(A) < T)) {
          x1 = -1;
        }
      }
      if (x0 <= x1) {
        const int rb = g.nx * (y + g.ny * z);
        pa = g.start[rb + x0];
        pb = g.start[rb + x1 + 1];
      }
    }
    // the 64 rows' ranges as chunks of 64 points, processed by the whole
    // wave (coalesced): chunk numbering by an inclusive scan of the rows'
    // chunk counts, chunk -> row by a binary search over the lanes
    const int nch = (pb - pa + 63) >> 6;
    int incl = nch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    const int excl = incl - nch;
    const int C = __shfl(incl, 63, 64);
    int acc = 0;
    for (int cb = 0; cb < C; cb += 64) {
      const int cc = cb + lane;
      int j = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const int e = __shfl(excl, min(j + step, 63), 64);
        if (j + step < 64 && e <= cc) j += step;
      }
      const int rbase = __shfl(pa, j, 64), rexcl = __shfl(excl, j, 64), rend = __shfl(pb, j, 64);
      const int cbase = cc < C ? rbase + (cc - rexcl) * 64 : 0;
      const int cend = cc < C ? rend : 0;
      const int nk = min(64, C - cb);
#pragma unroll 4
      for (int k = 0; k < nk; ++k) {
        const int base = __builtin_amdgcn_readlane(cbase, k), end = __builtin_amdgcn_readlane(cend, k);
        const int p = base + lane;
        if (p < end) {
          const float4 v = g.pts[p];
          const float dd = fmaf(P.x, v.x, fmaf(P.y, v.y, fmaf(P.z, v.z, P.w)));
          const float tt = fmaf(dd, dd, -Llo);
          if (tt < 0.0f) ++acc;
          else if (__float_as_uint(tt) <= wbits && plane_dist64(pl, v.x, v.y, v.z) < thr) ++acc;
        }
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0 && acc) atomicAdd(&counts32[h], acc);
  }
}

__global__ void k_counts_widen(const int32_t* __restrict__ c32, int H, int64_t* __restrict__ counts) {
  int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h < H) counts[h] = c32[h];
}

__global__ void k_mark_degenerate(const uint8_t* __restrict__ degenerate, int H, int64_t* __restrict__ counts) {
  int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h < H && degenerate[h]) counts[h] = -1;
}

constexpr int kSumBlocksX = 64;

__global__ void __launch_bounds__(kBlock) k_plane_abs_sum(const float* __restrict__ xyz, int64_t n,
                                                          const double* __restrict__ pl64, double thr,
                                                          double* __restrict__ partial) {
  __shared__ double sh[kBlock / 64];
  const double* pl = pl64 + 4 * blockIdx.y;
  const P3* p = reinterpret_cast<const P3*>(xyz);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    P3 q = p[i];
    double d = plane_dist64(pl, q.x, q.y, q.z);
    if (d < thr) acc += d;
  }
  double r = block_sum_f64<kBlock>(acc, sh);
  if (threadIdx.x == 0) partial[blockIdx.y * gridDim.x + blockIdx.x] = r;
}

__global__ void __launch_bounds__(kBlock) k_plane_flags(const float* __restrict__ xyz, int64_t n, double a, double b,
                                                        double c, double d, double thr, uint8_t* __restrict__ flags) {
  const double pl[4] = {a, b, c, d};
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    P3 q = p[i];
    flags[i] = plane_dist64(pl, q.x, q.y, q.z) < thr ? 1 : 0;
  }
}

constexpr int kMomBlocks = 256;

// pass 1 (centroid == nullptr): {x, y, z}; pass 2: centred {xx, xy, xz, yy, yz, zz}
__global__ void __launch_bounds__(kBlock) k_plane_moments(const float* __restrict__ xyz, const int32_t* __restrict__ idx,
                                                          int64_t m, double cx, double cy, double cz, int pass2,
                                                          double* __restrict__ partial) {
  __shared__ double sh[kBlock / 64];
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    int64_t i = idx ? idx[j] : j;
    double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (!pass2) {
      acc[0] += x;
      acc[1] += y;
      acc[2] += z;
    } else {
      double r0 = x - cx, r1 = y - cy, r2 = z - cz;
      acc[0] += r0 * r0;
      acc[1] += r0 * r1;
      acc[2] += r0 * r2;
      acc[3] += r1 * r1;
      acc[4] += r1 * r2;
      acc[5] += r2 * r2;
    }
  }
  for (int k = 0; k < 6; ++k) {
    double r = block_sum_f64<kBlock>(acc[k], sh);
    if (threadIdx.x == 0) partial[blockIdx.x * 6 + k] = r;
  }
}

__global__ void k_gather_samples(const float* __restrict__ xyz, const int32_t* __restrict__ idx, int64_t m,
                                 float* __restrict__ out) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  int64_t i = idx[j];
  out[3 * j] = xyz[3 * i];
  out[3 * j + 1] = xyz[3 * i + 1];
  out[3 * j + 2] = xyz[3 * i + 2];
}

// --------------------------------------------------------------- host math
static inline void hcross(const double u[3], const double v[3], double o[3]) {
  o[0] = u[1] * v[2] - u[2] * v[1];
  o[1] = u[2] * v[0] - u[0] * v[2];
  o[2] = u[0] * v[1] - u[1] * v[0];
}
static inline double hdot(const double u[3], const double v[3]) { return (u[0] * v[0] + u[1] * v[1]) + u[2] * v[2]; }

static void plane_from_centred(const double c[3], const double mo[6], double pl[4]) {
  const double xx = mo[0], xy = mo[1], xz = mo[2], yy = mo[3], yz = mo[4], zz = mo[5];
  double det_x = yy * zz - yz * yz, det_y = xx * zz - xz * xz, det_z = xx * yy - xy * xy;
  double abc[3];
  if (det_x > det_y && det_x > det_z) {
    abc[0] = det_x; abc[1] = xz * yz - xy * zz; abc[2] = xy * yz - xz * yy;
  } else if (det_y > det_z) {
    abc[0] = xz * yz - xy * zz; abc[1] = det_y; abc[2] = xy * xz - yz * xx;
  } else {
    abc[0] = xy * yz - xz * yy; abc[1] = xy * xz - yz * xx; abc[2] = det_z;
  }
  double norm = std::sqrt(hdot(abc, abc));
  if (norm == 0) {
    pl[0] = pl[1] = pl[2] = pl[3] = 0;
    return;
  }
  for (int a = 0; a < 3; ++a) abc[a] /= norm;
  pl[0] = abc[0]; pl[1] = abc[1]; pl[2] = abc[2];
  pl[3] = -hdot(abc, c);
}

// ComputeTrianglePlane (k == 3) / GetPlaneFromPoints (k > 3), host float64
static void plane_from_pts(const double* P, int k, double pl[4]) {
  if (k == 3) {
    double e0[3] = {P[3] - P[0], P[4] - P[1], P[5] - P[2]};
    double e1[3] = {P[6] - P[0], P[7] - P[1], P[8] - P[2]};
    double abc[3];
    hcross(e0, e1, abc);
    double norm = std::sqrt(hdot(abc, abc));
    if (norm == 0) {
      pl[0] = pl[1] = pl[2] = pl[3] = 0;
      return;
    }
    for (int a = 0; a < 3; ++a) abc[a] /= norm;
    pl[0] = abc[0]; pl[1] = abc[1]; pl[2] = abc[2];
    pl[3] = -hdot(abc, P);
    return;
  }
  double c[3] = {0, 0, 0};
  for (int j = 0; j < k; ++j)
    for (int a = 0; a < 3; ++a) c[a] += P[3 * j + a];
  for (int a = 0; a < 3; ++a) c[a] /= (double)k;
  double mo[6] = {0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    double r0 = P[3 * j] - c[0], r1 = P[3 * j + 1] - c[1], r2 = P[3 * j + 2] - c[2];
    mo[0] += r0 * r0; mo[1] += r0 * r1; mo[2] += r0 * r2;
    mo[3] += r1 * r1; mo[4] += r1 * r2; mo[5] += r2 * r2;
  }
  plane_from_centred(c, mo, pl);
}

static bool plane_is_zero(const double* pl) { return pl[0] == 0 && pl[1] == 0 && pl[2] == 0 && pl[3] == 0; }

// ------------------------------------------------------------ workspaces

// count geometry: nwp ranges of bpw batches of `batch` points
static void count_geometry(int64_t n, int batch, int* nwp, int64_t* bpw) {
  const int64_t nb = std::max<int64_t>(1, (n + batch - 1) / batch);
  *nwp = (int)std::min<int64_t>(kCountWaves, nb);
  *bpw = (nb + *nwp - 1) / *nwp;
}

// window bitmap: one word per (batch, chunk of hc hypotheses)
static int64_t count_flag_words(int64_t n, int H, int batch, int hc) {
  return std::max<int64_t>(1, (n + batch - 1) / batch) * ((std::max(H, 1) + hc - 1) / hc);
}

static int count_blocks(int64_t n) {
  int64_t tiles = (n + (int64_t)kBlock * kPts - 1) / ((int64_t)kBlock * kPts);
  return (int)std::max<int64_t>(1, std::min<int64_t>(kCountBlocksMax, tiles));
}

struct CountWs {
  float4* pl32;
  float4* band;
  double* pl64;
  uint8_t* degen;
  int32_t* partial;
  uint32_t* flags;  // (batch, hypothesis chunk) window bitmap of the brute-force count
  int32_t* counts32;
  void* grid_ws;    // cell grid of the cloud (the default count)
  size_t grid_ws_bytes;
  int64_t* counts;
  double* sum_partial;
  double* sums;
};

static size_t count_carve(Arena& ar, int64_t n, int H, CountWs* w) {
  H = std::max(H, 1);
  w->pl32 = ar.take<float4>(H);
  w->band = ar.take<float4>(H);
  w->pl64 = ar.take<double>(4 * (size_t)H);
  w->degen = ar.take<uint8_t>(H);
  w->partial = ar.take<int32_t>((size_t)std::max(count_blocks(n), kCountWaves) * H);
  w->flags = ar.take<uint32_t>((size_t)count_flag_words(n, H, kMinBatchPts, kMinHC));
  w->counts32 = ar.take<int32_t>(H);
  w->grid_ws_bytes = grid_ws_bytes(std::max<int64_t>(n, 1));
  w->grid_ws = ar.take<char>(w->grid_ws_bytes);
  w->counts = ar.take<int64_t>(H);
  w->sum_partial = ar.take<double>((size_t)kSumBlocksX * H);
  w->sums = ar.take<double>(H);
  return ar.used;
}

// scale of |a x| + |b y| + |c z| + |d| over the cloud, for the float32 band
static void upload_planes(const double* planes, int H, const double absmax[3], double thr, CountWs& w,
                          std::vector<float4>& p32, std::vector<float4>& bnd, std::vector<uint8_t>& dg,
                          hipStream_t s, int* rc) {
  p32.resize(H);
  bnd.resize(H);
  dg.resize(H);
  for (int h = 0; h < H; ++h) {
    const double* pl = planes + 4 * h;
    dg[h] = plane_is_zero(pl) ? 1 : 0;
    p32[h] = make_float4((float)pl[0], (float)pl[1], (float)pl[2], (float)pl[3]);
    double S = std::fabs(pl[0]) * absmax[0] + std::fabs(pl[1]) * absmax[1] + std::fabs(pl[2]) * absmax[2] +
               std::fabs(pl[3]);
    // float32 error of the fma chain: the four coefficients rounded (2^-24 S)
    // + three fma roundings (each <= 2^-24 S); 6 for margin, + 2^-20 thr for
    // the float32 rounding of lo / hi and Open3D's own float64 rounding
    double g = 6.0 * std::ldexp(1.0, -24) * S + std::ldexp(1.0, -20) * thr;
    float lo = (float)(thr - g), hi = (float)(thr + g);
    if (dg[h]) {
      lo = -1.0f;  // never an inlier
      hi = -1.0f;
    }
    // detection window mid +- half, covering [lo, hi) after float32 rounding
    // of |e - mid| (half widened by 2^-18 relative)
    const float mid = (float)(0.5 * ((double)lo + (double)hi));
    float half = (float)(std::max((double)mid - (double)lo, (double)hi - (double)mid) * (1.0 + std::ldexp(1.0, -18)));
    if (dg[h]) half = -1.0f;
    bnd[h] = make_float4(lo, hi, mid, half);
  }
  *rc = 0;
  if (hipMemcpyAsync(w.pl32, p32.data(), H * sizeof(float4), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(w.band, bnd.data(), H * sizeof(float4), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(w.pl64, planes, 4 * H * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(w.degen, dg.data(), H, hipMemcpyHostToDevice, s) != hipSuccess)
    *rc = fail(O3DX_EIO, "plane upload failed");
}

static int absmax_of(const float* xyz, int64_t n, void* aabb_ws, double* mm_dev, hipStream_t s, double out[3]) {
  double mm[6];
  O3DX_TRY(aabb_device(xyz, n, mm_dev, aabb_ws, s));
  O3DX_TRY(read_back(mm, mm_dev, 6 * sizeof(double), s));
  for (int a = 0; a < 3; ++a) out[a] = std::max(std::fabs(mm[a]), std::fabs(mm[3 + a]));
  return 0;
}

static int run_count(const float* xyz, int64_t n, const double* planes, int H, double thr, CountWs& w, void* aabb_ws,
                     double* mm_dev, hipStream_t s, std::vector<int64_t>& counts) {
  double absmax[3];
  O3DX_TRY(absmax_of(xyz, n, aabb_ws, mm_dev, s, absmax));
  std::vector<float4> p32;
  std::vector<float4> bnd;
  std::vector<uint8_t> dg;
  int rc;
  upload_planes(planes, H, absmax, thr, w, p32, bnd, dg, s, &rc);
  if (rc) return rc;
  int nb = count_blocks(n);
  KTimer kt("plane_count", s);
  if (!getenv("O3DX_RANSAC_VALU")) {
    // one window for all hypotheses: the union of their float32 windows
    // (degenerate and non-finite planes are never counted: left out)
    float lo = -1.0f, hi = -1.0f;
    bool any = false;
    for (int h = 0; h < H; ++h)
      if (!dg[h] && std::isfinite(bnd[h].x) && std::isfinite(bnd[h].y)) {
        lo = any ? std::min(lo, bnd[h].x) : bnd[h].x;
        hi = any ? std::max(hi, bnd[h].y) : bnd[h].y;
        any = true;
      }
    // squares: Llo <= lo^2 (rounded down; 0 when lo <= 0 or tiny: nothing is
    // certain), Lhi >= hi^2 (rounded up), window bits(t) <= bits(fl(Lhi - Llo)):
    // d^2 < Lhi => t = fl(d^2 - Llo) <= fl(Lhi - Llo) (rounding is monotone)
    auto f32_down = [](double v) { float f = (float)v; return (double)f > v ? std::nextafter(f, -INFINITY) : f; };
    auto f32_up = [](double v) { float f = (float)v; return (double)f < v ? std::nextafter(f, INFINITY) : f; };
    const double lo2 = (double)lo * (double)lo, hi2 = (double)hi * (double)hi;
    const float Llo = (lo > 0.0f && lo2 > std::ldexp(1.0, -100)) ? f32_down(lo2) : 0.0f;
    const float Lhi = hi > 0.0f ? f32_up(hi2) : 0.0f;
    const float wdt = (float)((double)Lhi - (double)Llo);  // exact difference, one rounding
    uint32_t wbits;
    std::memcpy(&wbits, &wdt, 4);
    if (!getenv("O3DX_RANSAC_BRUTE")) {
      // cell grid of the cloud: whole cells decided per hypothesis
      GridBuild G;
      const double occ = getenv("O3DX_RANSAC_OCC") ? atof(getenv("O3DX_RANSAC_OCC")) : 48.0;
      O3DX_TRY(grid_build(xyz, n, occ, 0.0, w.grid_ws, w.grid_ws_bytes, s, &G, nullptr, nullptr, false, 4,
                          /*ordered=*/false));
      const GridView& g = G.view;
      const double hh = g.h, amax = std::max(std::max(absmax[0], absmax[1]), absmax[2]);
      // float64 rounding of a cell-centre distance and of Open3D's distance
      const double cmargin = 64.0 * std::ldexp(1.0, -52) * (3.0 * (amax + 4 * hh) + amax + 1.0) * 2.0 + 1e-12 * thr;
      const int rows = g.ny * g.nz;
      const int gph = (rows + 63) / 64;  // 64-row groups per hypothesis
      const int64_t tasks = (int64_t)H * gph;
      O3DX_HIP(hipMemsetAsync(w.counts32, 0, (size_t)H * sizeof(int32_t), s));
      hipLaunchKernelGGL(k_plane_count_grid, dim3(grid_for(tasks, kBlock / 64, 16384)), dim3(kBlock), 0, s, g,
                         w.pl32, w.pl64, H, thr, Llo, wbits, cmargin, gph, w.counts32);
      hipLaunchKernelGGL(k_counts_widen, dim3((H + 255) / 256), dim3(256), 0, s, w.counts32, H, w.counts);
      hipLaunchKernelGGL(k_mark_degenerate, dim3((H + 255) / 256), dim3(256), 0, s, w.degen, H, w.counts);
      kt.stop();
      counts.resize(H);
      O3DX_TRY(read_back(counts.data(), w.counts, H * sizeof(int64_t), s));
      O3DX_HIP(hipGetLastError());
      return 0;
    }
    // brute force: every point against every hypothesis
    int hc = 32, pl = 16;
    if (const char* e = getenv("O3DX_RANSAC_SHAPE")) sscanf(e, "%dx%d", &hc, &pl);
    int nwp;
    int64_t bpw;
    count_geometry(n, 64 * pl, &nwp, &bpw);
    const int nchunks = (H + hc - 1) / hc;
    const int ncg = (nchunks + kBlock / 64 - 1) / (kBlock / 64);  // blocks per batch range
    const int64_t nwords = count_flag_words(n, H, 64 * pl, hc);
    const unsigned fgrid = grid_for(nwords, kBlock / 64, 16384);
#define O3DX_COUNT(HC, PL)                                                                                         \
  if (hc == HC && pl == PL) {                                                                                      \
    hipLaunchKernelGGL((k_plane_count_v<HC, PL>), dim3((unsigned)(nwp * ncg)), dim3(kBlock), 0, s, xyz, n, w.pl32, \
                       H, Llo, wbits, bpw, nwp, ncg, w.partial, w.flags);                                          \
    O3DX_TRY(reduce_columns_i32_to_i64(w.partial, nwp, H, w.counts, s));                                          \
    hipLaunchKernelGGL((k_plane_fixup<HC, PL>), dim3(fgrid), dim3(kBlock), 0, s, xyz, n, w.pl32, w.pl64, H, thr,   \
                       Llo, wbits, w.flags, nwords, w.counts);                                                      \
  } else
    O3DX_COUNT(32, 16) O3DX_COUNT(32, 8) O3DX_COUNT(16, 16) O3DX_COUNT(16, 8)
    return fail(O3DX_EINVAL, "O3DX_RANSAC_SHAPE: instantiated shapes are 32x16, 32x8, 16x16, 16x8");
#undef O3DX_COUNT
  } else {  // the ballot/popcount kernel with per-hypothesis windows (A/B reference)
    for (int h0 = 0; h0 < H; h0 += kHChunk) {
      int hc = std::min(kHChunk, H - h0);
      hipLaunchKernelGGL(k_plane_count, dim3(nb), dim3(kBlock), 0, s, xyz, n, w.pl32, w.band, w.pl64, H, h0, hc, thr,
                         w.partial);
    }
    O3DX_TRY(reduce_columns_i32_to_i64(w.partial, nb, H, w.counts, s));
  }
  hipLaunchKernelGGL(k_mark_degenerate, dim3((H + 255) / 256), dim3(256), 0, s, w.degen, H, w.counts);
  kt.stop();
  counts.resize(H);
  O3DX_TRY(read_back(counts.data(), w.counts, H * sizeof(int64_t), s));
  O3DX_HIP(hipGetLastError());
  return 0;
}

static int run_abs_sum(const float* xyz, int64_t n, const double* planes, const int32_t* which, int L, double thr,
                       CountWs& w, hipStream_t s, double* sums_host) {
  if (L == 0) return 0;
  std::vector<double> sel((size_t)4 * L);
  for (int j = 0; j < L; ++j)
    for (int a = 0; a < 4; ++a) sel[4 * j + a] = planes[4 * which[j] + a];
  O3DX_HIP(hipMemcpyAsync(w.pl64, sel.data(), sel.size() * sizeof(double), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_plane_abs_sum, dim3(kSumBlocksX, L), dim3(kBlock), 0, s, xyz, n, w.pl64, thr, w.sum_partial);
  // fixed-order final sums on the host
  std::vector<double> part((size_t)kSumBlocksX * L);
  O3DX_TRY(read_back(part.data(), w.sum_partial, part.size() * sizeof(double), s));
  O3DX_HIP(hipGetLastError());
  for (int j = 0; j < L; ++j) {
    double t = 0.0;
    for (int b = 0; b < kSumBlocksX; ++b) t += part[(size_t)j * kSumBlocksX + b];
    sums_host[j] = t;
  }
  return 0;
}

static int select_best(const int64_t* counts, const double* sums, const double* planes, int H, int64_t n, int ransac_n,
                       double probability) {
  double best_fit = 0, best_rmse = 0;
  int best = -1;
  size_t break_iteration = std::numeric_limits<size_t>::max();
  int iteration_count = 0;
  for (int it = 0; it < H; ++it) {
    if ((size_t)iteration_count > break_iteration) continue;
    if (counts[it] < 0 || (planes && plane_is_zero(planes + 4 * it))) continue;
    double fit = counts[it] == 0 ? 0.0 : (double)counts[it] / (double)n;
    double rmse = counts[it] == 0 ? 0.0 : sums[it] / std::sqrt((double)counts[it]);
    if (fit > best_fit || (fit == best_fit && rmse < best_rmse)) {
      best_fit = fit;
      best_rmse = rmse;
      best = it;
      if (best_fit < 1.0) {
        double bi = std::min(std::log(1 - probability) / std::log(1 - std::pow(best_fit, ransac_n)), (double)H);
        break_iteration = (size_t)bi;
      } else {
        break_iteration = 0;
      }
    }
    iteration_count++;
  }
  return best;
}

// hypotheses whose count equals another non-degenerate hypothesis' count
static std::vector<int32_t> tied_hypotheses(const std::vector<int64_t>& counts) {
  std::vector<std::pair<int64_t, int32_t>> v;
  for (int h = 0; h < (int)counts.size(); ++h)
    if (counts[h] > 0) v.emplace_back(counts[h], h);
  std::sort(v.begin(), v.end());
  std::vector<int32_t> out;
  for (size_t i = 0; i < v.size(); ++i) {
    bool t = (i > 0 && v[i].first == v[i - 1].first) || (i + 1 < v.size() && v[i].first == v[i + 1].first);
    if (t) out.push_back(v[i].second);
  }
  std::sort(out.begin(), out.end());
  return out;
}

static int run_moments(const float* xyz, const int32_t* idx, int64_t m, const double* centroid, double* part,
                       double* out_dev, hipStream_t s, double out[6]) {
  if (m == 0) {
    for (int k = 0; k < 6; ++k) out[k] = 0;
    return 0;
  }
  const int nb = (int)std::min<int64_t>(kMomBlocks, (m + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_plane_moments, dim3(nb), dim3(kBlock), 0, s, xyz, idx, m, centroid ? centroid[0] : 0.0,
                     centroid ? centroid[1] : 0.0, centroid ? centroid[2] : 0.0, centroid ? 1 : 0, part);
  O3DX_TRY(reduce_columns_f64(part, nb, 6, out_dev, s));
  O3DX_TRY(read_back(out, out_dev, 6 * sizeof(double), s));
  O3DX_HIP(hipGetLastError());
  return 0;
}

struct SegWs {
  CountWs cw;
  int32_t* sidx;
  float* scoord;
  uint8_t* flags;
  int32_t* scan_tmp;
  char* aabb;
  double* mm;
  int64_t* cnt;
  double* mom_part;
  double* mom_out;
};

static size_t seg_carve(Arena& ar, int64_t n, int H, int rn, SegWs* w) {
  count_carve(ar, n, H, &w->cw);
  w->sidx = ar.take<int32_t>((size_t)H * rn);
  w->scoord = ar.take<float>((size_t)H * rn * 3);
  w->flags = ar.take<uint8_t>(n + 16);
  w->scan_tmp = ar.take<int32_t>(compact_workspace_ints(n));
  w->aabb = ar.take<char>(aabb_ws_bytes(n));
  w->mm = ar.take<double>(8);
  w->cnt = ar.take<int64_t>(4);
  w->mom_part = ar.take<double>(kMomBlocks * 6);
  w->mom_out = ar.take<double>(8);
  return ar.used;
}

}  // namespace o3dx

using namespace o3dx;

extern "C" int o3dx_ransac_samples(int64_t n, int ransac_n, int iters, uint64_t seed, int32_t* out) {
  if (n <= 0 || ransac_n <= 0 || iters < 0 || !out || n < ransac_n)
    return fail(O3DX_EINVAL, "o3dx_ransac_samples: need n >= ransac_n > 0");
  // Open3D RandomSampler: RandUint32() % total_size, redraw duplicates
  std::mt19937 eng((uint32_t)seed);
  for (int it = 0; it < iters; ++it) {
    int got = 0;
    while (got < ransac_n) {
      int32_t idx = (int32_t)((uint64_t)eng() % (uint64_t)n);
      bool dup = false;
      for (int j = 0; j < got; ++j) dup |= out[(int64_t)it * ransac_n + j] == idx;
      if (!dup) out[(int64_t)it * ransac_n + got++] = idx;
    }
  }
  return 0;
}

extern "C" int o3dx_plane_from_points(const double* pts, int k, double* plane) {
  if (!pts || !plane || k < 3) return fail(O3DX_EINVAL, "o3dx_plane_from_points: need k >= 3");
  plane_from_pts(pts, k, plane);
  return 0;
}

extern "C" int o3dx_plane_from_moments(const double* sum_xyz, int64_t count, const double* centred, double* plane) {
  if (!sum_xyz || !centred || !plane) return fail(O3DX_EINVAL, "o3dx_plane_from_moments: bad arguments");
  double c[3];
  for (int a = 0; a < 3; ++a) c[a] = sum_xyz[a] / (double)count;
  plane_from_centred(c, centred, plane);
  return 0;
}

extern "C" size_t o3dx_plane_count_workspace_bytes(int64_t n, int H) {
  Arena ar(nullptr, 0);
  CountWs w;
  count_carve(ar, std::max<int64_t>(n, 1), H, &w);
  return ar.used + Arena::align(aabb_ws_bytes(n)) + 1024;
}

extern "C" int o3dx_plane_count(const float* xyz, int64_t n, const double* planes, int H, double thr, int64_t* counts,
                                void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || H < 0 || (n > 0 && !xyz) || (H > 0 && (!planes || !counts)))
    return fail(O3DX_EINVAL, "o3dx_plane_count: bad arguments");
  if (!ws || ws_bytes < o3dx_plane_count_workspace_bytes(n, H)) return fail(O3DX_ENOMEM, "plane_count workspace too small");
  if (H == 0) return 0;
  if (n == 0) {
    for (int h = 0; h < H; ++h) counts[h] = plane_is_zero(planes + 4 * h) ? -1 : 0;
    return 0;
  }
  hipStream_t s = as_stream(stream);
  Arena ar(ws, ws_bytes);
  CountWs w;
  count_carve(ar, n, H, &w);
  char* aabb = ar.take<char>(aabb_ws_bytes(n));
  double* mm = ar.take<double>(8);
  O3DX_ARENA_CHECK(ar);
  std::vector<int64_t> c;
  O3DX_TRY(run_count(xyz, n, planes, H, thr, w, aabb, mm, s, c));
  std::memcpy(counts, c.data(), H * sizeof(int64_t));
  return 0;
}

extern "C" int o3dx_plane_abs_sum(const float* xyz, int64_t n, const double* planes, const int32_t* which, int L,
                                  double thr, double* sums, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || L < 0 || (L > 0 && (!planes || !which || !sums))) return fail(O3DX_EINVAL, "o3dx_plane_abs_sum: bad args");
  if (!ws || ws_bytes < o3dx_plane_count_workspace_bytes(n, L)) return fail(O3DX_ENOMEM, "abs_sum workspace too small");
  if (L == 0) return 0;
  if (n == 0) {
    for (int j = 0; j < L; ++j) sums[j] = 0;
    return 0;
  }
  Arena ar(ws, ws_bytes);
  CountWs w;
  count_carve(ar, n, L, &w);
  O3DX_ARENA_CHECK(ar);
  return run_abs_sum(xyz, n, planes, which, L, thr, w, as_stream(stream), sums);
}

extern "C" int o3dx_ransac_select(const int64_t* counts, const double* sums, const double* planes, int H, int64_t n,
                                  int ransac_n, double probability) {
  if (!counts || !sums || H < 0 || n <= 0) return -1;
  return select_best(counts, sums, planes, H, n, ransac_n, probability);
}

extern "C" int o3dx_plane_inliers(const float* xyz, int64_t n, const double* plane, double thr, int32_t* idx_out,
                                  int64_t* count_host, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || !plane || !count_host || (n > 0 && (!xyz || !idx_out))) return fail(O3DX_EINVAL, "o3dx_plane_inliers: bad args");
  size_t need = Arena::align(n + 17) + Arena::align(compact_workspace_ints(n) * 4 + 1) + 512;
  if (!ws || ws_bytes < need) return fail(O3DX_ENOMEM, "plane_inliers workspace too small");
  if (n == 0 || plane_is_zero(plane)) {
    *count_host = 0;
    return 0;
  }
  hipStream_t s = as_stream(stream);
  Arena ar(ws, ws_bytes);
  uint8_t* flags = ar.take<uint8_t>(n + 16);
  int32_t* tmp = ar.take<int32_t>(compact_workspace_ints(n));
  int64_t* cnt = ar.take<int64_t>(2);
  hipLaunchKernelGGL(k_plane_flags, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, plane[0], plane[1],
                     plane[2], plane[3], thr, flags);
  O3DX_TRY(compact_flags(flags, n, idx_out, nullptr, cnt, tmp, s));
  O3DX_TRY(read_back(count_host, cnt, sizeof(int64_t), s));
  return 0;
}

extern "C" int o3dx_plane_moments(const float* xyz, const int32_t* idx, int64_t count, const double* centroid,
                                  double* sums, void* ws, size_t ws_bytes, void* stream) {
  if (count < 0 || !sums || (count > 0 && !xyz)) return fail(O3DX_EINVAL, "o3dx_plane_moments: bad args");
  if (!ws || ws_bytes < 8192 + kMomBlocks * 6 * sizeof(double)) return fail(O3DX_ENOMEM, "moments workspace too small");
  Arena ar(ws, ws_bytes);
  double* part = ar.take<double>(kMomBlocks * 6);
  double* outd = ar.take<double>(8);
  double tmp[6];
  O3DX_TRY(run_moments(xyz, idx, count, centroid, part, outd, as_stream(stream), tmp));
  std::memcpy(sums, tmp, (centroid ? 6 : 3) * sizeof(double));
  return 0;
}

extern "C" size_t o3dx_segment_plane_workspace_bytes(int64_t n, int iters) {
  Arena ar(nullptr, 0);
  SegWs w;
  // ransac_n up to 16 sample points per hypothesis in the sample buffers
  seg_carve(ar, std::max<int64_t>(n, 1), std::max(iters, 1), 16, &w);
  return ar.used + 1024;
}

extern "C" int o3dx_segment_plane(const float* xyz, int64_t n, double thr, int ransac_n, int iters, double probability,
                                  const int32_t* samples_host, double* plane_host, int32_t* inliers_out,
                                  int64_t* n_inliers_host, void* ws, size_t ws_bytes, void* stream) {
  if (!(probability > 0.0 && probability <= 1.0)) return fail(O3DX_EINVAL, "Probability must be > 0 or <= 1.0");
  if (ransac_n < 3) return fail(O3DX_EINVAL, "ransac_n should be set to higher than or equal to 3.");
  if (n < ransac_n) return fail(O3DX_EINVAL, "There must be at least 'ransac_n' points.");
  if (ransac_n > 16) return fail(O3DX_ENOTSUP, "ransac_n > 16 not supported");
  if (iters < 0 || !plane_host || !n_inliers_host || !inliers_out || !xyz || (iters > 0 && !samples_host))
    return fail(O3DX_EINVAL, "o3dx_segment_plane: bad arguments");
  if (!ws || ws_bytes < o3dx_segment_plane_workspace_bytes(n, iters))
    return fail(O3DX_ENOMEM, "segment_plane workspace too small");
  hipStream_t s = as_stream(stream);
  Arena ar(ws, ws_bytes);
  SegWs w;
  seg_carve(ar, n, std::max(iters, 1), 16, &w);
  const int H = iters;
  // hypotheses (host float64, from the sampled points' coordinates)
  std::vector<double> planes((size_t)4 * std::max(H, 1), 0.0);
  if (H > 0) {
    const int64_t ns = (int64_t)H * ransac_n;
    for (int64_t j = 0; j < ns; ++j)
      if (samples_host[j] < 0 || samples_host[j] >= n) return fail(O3DX_EINVAL, "sample index out of range");
    O3DX_HIP(hipMemcpyAsync(w.sidx, samples_host, ns * sizeof(int32_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_gather_samples, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, xyz, w.sidx, ns, w.scoord);
    std::vector<float> sc((size_t)ns * 3);
    O3DX_TRY(read_back(sc.data(), w.scoord, sc.size() * sizeof(float), s));
    std::vector<double> P((size_t)ransac_n * 3);
    for (int h = 0; h < H; ++h) {
      for (int j = 0; j < ransac_n * 3; ++j) P[j] = (double)sc[(size_t)h * ransac_n * 3 + j];
      plane_from_pts(P.data(), ransac_n, &planes[(size_t)4 * h]);
    }
  }
  int best = -1;
  if (H > 0) {
    std::vector<int64_t> counts;
    O3DX_TRY(run_count(xyz, n, planes.data(), H, thr, w.cw, w.aabb, w.mm, s, counts));
    std::vector<int32_t> tied = tied_hypotheses(counts);
    std::vector<double> sums(H, std::numeric_limits<double>::quiet_NaN());
    if (!tied.empty()) {
      std::vector<double> ts(tied.size());
      O3DX_TRY(run_abs_sum(xyz, n, planes.data(), tied.data(), (int)tied.size(), thr, w.cw, s, ts.data()));
      for (size_t j = 0; j < tied.size(); ++j) sums[tied[j]] = ts[j];
    }
    best = select_best(counts.data(), sums.data(), planes.data(), H, n, ransac_n, probability);
  }
  double bp[4] = {0, 0, 0, 0};
  if (best >= 0) std::memcpy(bp, &planes[(size_t)4 * best], sizeof(bp));
  int64_t k = 0;
  if (!plane_is_zero(bp)) {
    hipLaunchKernelGGL(k_plane_flags, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, bp[0], bp[1], bp[2],
                       bp[3], thr, w.flags);
    O3DX_TRY(compact_flags(w.flags, n, inliers_out, nullptr, w.cnt, w.scan_tmp, s));
    O3DX_TRY(read_back(&k, w.cnt, sizeof(int64_t), s));
  }
  *n_inliers_host = k;
  // GetPlaneFromPoints over the final inliers (zero plane when there are none)
  if (k == 0) {
    for (int a = 0; a < 4; ++a) plane_host[a] = 0;
    return 0;
  }
  double s1[6], s2[6], c[3];
  O3DX_TRY(run_moments(xyz, inliers_out, k, nullptr, w.mom_part, w.mom_out, s, s1));
  for (int a = 0; a < 3; ++a) c[a] = s1[a] / (double)k;
  O3DX_TRY(run_moments(xyz, inliers_out, k, c, w.mom_part, w.mom_out, s, s2));
  plane_from_centred(c, s2, plane_host);
  return 0;
}
