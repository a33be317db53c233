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
#include <cfloat>
#include <cstring>
#include <random>
#include <vector>

#include "common.hpp"

namespace o3dx {

constexpr int kPts = 16;
constexpr int kCountBlocksMax = 4096;

struct P3 {
  float x, y, z;
};

// a point's coordinates as float64: a float32 cloud's (exact) or a float64 cloud's own
__device__ __forceinline__ void load3(const float* xyz, int64_t i, double& x, double& y, double& z) {
  const P3 q = reinterpret_cast<const P3*>(xyz)[i];
  x = q.x;
  y = q.y;
  z = q.z;
}
__device__ __forceinline__ void load3(const double* xyz, int64_t i, double& x, double& y, double& z) {
  x = xyz[3 * i];
  y = xyz[3 * i + 1];
  z = xyz[3 * i + 2];
}

__device__ __forceinline__ double plane_dist64(const double* pl, double x, double y, double z) {
  // Eigen Vector4d dot packet order: (a*x + c*z) + (b*y + d*1)
  double ax = pl[0] * x, by = pl[1] * y, cz = pl[2] * z, dw = pl[3] * 1.0;
  return fabs((ax + cz) + (by + dw));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

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
// 64 PL points): 32 x 16 at 6 waves per SIMD, and for the exact rounds'
// few hypotheses 16 x 16 / 8 x 16 at 8 waves.
constexpr int kCountWaves = 2048;      // batch ranges (waves per hypothesis chunk)
constexpr int kMinBatchPts = 64 * 8;   // smallest instantiated batch (bitmap sizing)
constexpr int kMinHC = 8;              // smallest instantiated chunk (bitmap sizing)

template <int PL>
__device__ __forceinline__ void plane_batch_load(const P3* __restrict__ p, int64_t n, int64_t gb, int lane,
                                                 f32x2 (&X)[PL / 2], f32x2 (&Y)[PL / 2], f32x2 (&Z)[PL / 2]) {
  const float qnan = __int_as_float(0x7fc00000);
  // wave-uniform batch base and remainder; 32-bit lane offsets (saddr form)
  const P3* base = p + gb * (64 * PL);
  const int64_t rem64 = n - gb * (64 * PL);
  const uint32_t rem = (uint32_t)min<int64_t>(rem64, 64 * PL);
#pragma unroll
  for (int k = 0; k < PL / 2; ++k) {
    const uint32_t i0 = (uint32_t)(2 * k) * 64 + lane, i1 = i0 + 64;
    // clamped, unconditional loads; rows past n become NaN afterwards
    const P3 a = base[min(i0, rem - 1)];
    const P3 b = base[min(i1, rem - 1)];
    X[k] = (f32x2){i0 < rem ? a.x : qnan, i1 < rem ? b.x : qnan};
    Y[k] = (f32x2){i0 < rem ? a.y : qnan, i1 < rem ? b.y : qnan};
    Z[k] = (f32x2){i0 < rem ? a.z : qnan, i1 < rem ? b.z : qnan};
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

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// block -> (batch range, group of 4 hypothesis chunks), XCD-aware: the
// launch's blocks are dealt round-robin over the 8 XCDs, so logical block
// l = (b % 8) * (nb / 8) + b / 8 puts consecutive l on one XCD.
__device__ __forceinline__ int xcd_logical_block(int b, int nb) {
  if (nb % 8) return b;
  return (b % 8) * (nb / 8) + b / 8;
}

// Per hypothesis of the chunk the wave keeps its count in a scalar register
// across the whole batch range (popcounts summed on the scalar unit), so the
// per-batch work is exactly: 4 v_readlane (the plane), PL/2 x (3 + 1) packed
// fmas, PL compares, PL/2 v_min3 and one window ballot.  PF: the next batch's
// points are loaded while the current one is evaluated.
template <int kHC, int kPL, int kPF>  // kHC <= 32: one bitmap bit per hypothesis
__device__ __forceinline__ void plane_count_body(const float* __restrict__ xyz, int64_t n,
                                                 const float4* __restrict__ pl32, int H, float Llo, uint32_t wbits,
                                                 int64_t batches_per_wave, int nwp, int ncg,
                                                 int32_t* __restrict__ partial, uint32_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int wp = lb / ncg;                                                      // batch range
  const int chunk = __builtin_amdgcn_readfirstlane((lb % ncg) * (kBlock / 64) + (threadIdx.x >> 6));
  const int nchunks = (H + kHC - 1) / kHC;
  if (wp >= nwp || chunk >= nchunks) return;
  const int h0 = chunk * kHC;
  const P3* p = reinterpret_cast<const P3*>(xyz);
  int sc[kHC];  // wave-uniform counts of hypotheses h0 .. h0 + kHC
#pragma unroll
  for (int h = 0; h < kHC; ++h) sc[h] = 0;
  // lane j holds plane h0 + (j % kHC) (h0 + j >= H: a copy of the last plane,
  // its counts never written back)
  float4 Pl = pl32[min(h0 + (lane % kHC), H - 1)];
  constexpr int kBatchPts = 64 * kPL;
  const int64_t nbatches = (n + kBatchPts - 1) / kBatchPts;
  const int64_t gb0 = (int64_t)wp * batches_per_wave;
  const int64_t gbe = min(gb0 + batches_per_wave, nbatches);
  f32x2 X[kPL / 2], Y[kPL / 2], Z[kPL / 2];
  if (kPF && gb0 < gbe) plane_batch_load<kPL>(p, n, gb0, lane, X, Y, Z);
  for (int64_t gb = gb0; gb < gbe; ++gb) {
    if (!kPF) plane_batch_load<kPL>(p, n, gb, lane, X, Y, Z);
    f32x2 Xn[kPL / 2], Yn[kPL / 2], Zn[kPL / 2];
    if (kPF && gb + 1 < gbe) plane_batch_load<kPL>(p, n, gb + 1, lane, Xn, Yn, Zn);
    // the planes are read out of Pl per batch, not hoisted out of the batch
    // loop into 128 scalar registers (an empty asm that "changes" Pl)
    asm volatile("" : "+v"(Pl.x), "+v"(Pl.y), "+v"(Pl.z), "+v"(Pl.w));
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
      int c = 0;  // wave-uniform
#pragma unroll
      for (int k = 0; k < kPL / 2; ++k) {
        const f32x2 t = plane_sq_test(plane_dist_pk(P, X[k], Y[k], Z[k]), Llo);
        // inliers: one v_cmp per point, counted on the scalar unit
        c += __popcll(__ballot(t.x < 0.0f)) + __popcll(__ballot(t.y < 0.0f));
        asm("" : "+s"(c));  // summed as they come (a deferred sum tree spills the masks)
        mn = umin3(mn, __float_as_uint(t.x), __float_as_uint(t.y));
      }
      sc[h] += c;
      if (__ballot(mn <= wbits)) word |= 1u << h;
    }
    if (lane == 0) flags[gb * nchunks + chunk] = word;
    if (kPF && gb + 1 < gbe) {
#pragma unroll
      for (int k = 0; k < kPL / 2; ++k) {
        X[k] = Xn[k];
        Y[k] = Yn[k];
        Z[k] = Zn[k];
      }
    }
  }
  int mine = 0;
#pragma unroll
  for (int h = 0; h < kHC; ++h) mine = lane == h ? sc[h] : mine;
  if (lane < kHC && h0 + lane < H) partial[(int64_t)wp * H + h0 + lane] = mine;
}

// the register budget of 8 / 6 waves per SIMD (occupancy for the dependent
// fma -> compare -> popcount chains; measured r03: 2.4 ms at 4 waves, 1.5 at 6)
template <int kHC, int kPL, int kPF>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_plane_count_w8(const float* __restrict__ xyz, int64_t n, const float4* __restrict__ pl32, int H, float Llo,
                 uint32_t wbits, int64_t bpw, int nwp, int ncg, int32_t* __restrict__ partial,
                 uint32_t* __restrict__ flags) {
  plane_count_body<kHC, kPL, kPF>(xyz, n, pl32, H, Llo, wbits, bpw, nwp, ncg, partial, flags);
}
template <int kHC, int kPL, int kPF>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 6)))
k_plane_count_w6(const float* __restrict__ xyz, int64_t n, const float4* __restrict__ pl32, int H, float Llo,
                 uint32_t wbits, int64_t bpw, int nwp, int ncg, int32_t* __restrict__ partial,
                 uint32_t* __restrict__ flags) {
  plane_count_body<kHC, kPL, kPF>(xyz, n, pl32, H, Llo, wbits, bpw, nwp, ncg, partial, flags);
}

// Upper bounds of the counts (ub >= the exact count, bit-exactly so): a point
// is counted when its float32 |d| < hi, hi >= thr + g of every hypothesis
// (rounded up), so every float64 inlier is counted.  No window and no
// bitmap: per batch and hypothesis 4 v_readlane, PL/2 x 3 packed fmas and PL
// compares (|d| through the abs modifier).  segment_plane selects on these
// and counts exactly only the hypotheses its replay could consult
// (needed_exact below) — Open3D's records, typically ~ln H of H.
template <int kHC, int kPL>
__device__ __forceinline__ void plane_upper_body(const float* __restrict__ xyz, int64_t n,
                                                 const float4* __restrict__ pl32, int H, float hi,
                                                 int64_t batches_per_wave, int nwp, int ncg,
                                                 int32_t* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int wp = lb / ncg;
  const int chunk = __builtin_amdgcn_readfirstlane((lb % ncg) * (kBlock / 64) + (threadIdx.x >> 6));
  const int nchunks = (H + kHC - 1) / kHC;
  if (wp >= nwp || chunk >= nchunks) return;
  const int h0 = chunk * kHC;
  const P3* p = reinterpret_cast<const P3*>(xyz);
  int sc[kHC];
#pragma unroll
  for (int h = 0; h < kHC; ++h) sc[h] = 0;
  float4 Pl = pl32[min(h0 + (lane % kHC), H - 1)];
  constexpr int kBatchPts = 64 * kPL;
  const int64_t nbatches = (n + kBatchPts - 1) / kBatchPts;
  const int64_t gb0 = (int64_t)wp * batches_per_wave;
  const int64_t gbe = min(gb0 + batches_per_wave, nbatches);
  for (int64_t gb = gb0; gb < gbe; ++gb) {
    f32x2 X[kPL / 2], Y[kPL / 2], Z[kPL / 2];
    plane_batch_load<kPL>(p, n, gb, lane, X, Y, Z);
    asm volatile("" : "+v"(Pl.x), "+v"(Pl.y), "+v"(Pl.z), "+v"(Pl.w));
#pragma unroll
    for (int h = 0; h < kHC; ++h) {
      const float4 P = make_float4(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.x), h)),
                                   __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.y), h)),
                                   __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.z), h)),
                                   __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Pl.w), h)));
      int c = 0;
#pragma unroll
      for (int k = 0; k < kPL / 2; ++k) {
        const f32x2 d = plane_dist_pk(P, X[k], Y[k], Z[k]);
        c += __popcll(__ballot(fabsf(d.x) < hi)) + __popcll(__ballot(fabsf(d.y) < hi));
        asm("" : "+s"(c));  // summed as they come
      }
      sc[h] += c;
    }
  }
  int mine = 0;
#pragma unroll
  for (int h = 0; h < kHC; ++h) mine = lane == h ? sc[h] : mine;
  if (lane < kHC && h0 + lane < H) partial[(int64_t)wp * H + h0 + lane] = mine;
}

template <int kHC, int kPL>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 6)))
k_plane_upper(const float* __restrict__ xyz, int64_t n, const float4* __restrict__ pl32, int H, float hi,
              int64_t bpw, int nwp, int ncg, int32_t* __restrict__ partial) {
  plane_upper_body<kHC, kPL>(xyz, n, pl32, H, hi, bpw, nwp, ncg, partial);
}

// Upper bounds on the matrix cores.  The distances of 32 points to 32
// hypotheses are v_mfma_f32_32x32x16_bf16 products of bf16 parts (round to
// nearest) of the float32 coordinates and the float64 coefficients; bf16 x
// bf16 products are exact in float32.
//  TIGHT = false, one MFMA (K = 16), two parts each (x = xh + xl + xr,
//    |xr| <= 2^-16 |x|):
//      xh.ah + yh.bh + zh.ch + dh | xl.ah + yl.bh + zl.ch + dl | xh.al + yh.bl + zh.cl
//    dropped xl.al, xr.a, x.ar, dr (<= 3.1 2^-16 S) + float32 accumulation of
//    11 terms (<= 2^-19.5 S): |error| < 2^-14 S_h.
//  TIGHT = true, two MFMAs (K = 32), three parts each (the float32 coordinate
//    exactly: 3 x 8 significant bits; |ar| <= 2^-24 |a|):
//      h.h, h.m, m.h, m.m, h.l, l.h per coordinate + dh + dm + dl
//    dropped m.l, l.m, l.l, x.ar, dr (<= 3.1 2^-24 S) + float32 accumulation of
//    21 terms (<= 2^-18.4 S): |error| < 2^-17 S_h.
// S_h = |a| max|x| + |b| max|y| + |c| max|z| + |d|.  Counting |d| < hi_h, hi_h
// >= thr + (that bound) counts every float64 inlier: an upper bound, as
// k_plane_upper's (whose float32 band is 6 2^-24 S_h + 2^-20 thr).  The result
// tile has the hypothesis on the lane (column lane & 31) and 16 point rows in
// the registers: one compare + one add-with-carry per element, a count per
// lane, no ballots or scalar popcounts (k_plane_upper's VALU distances cost
// 1.5 packed fmas + a compare per pair: twice the issue).  Rows past n are
// NaN: never counted.
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
template <bool TIGHT>
struct MfmaShape {
  static constexpr int kTiles = TIGHT ? 4 : 8;      // 32-point tiles per wave batch (A fragments in registers)
  static constexpr int kChunks = TIGHT ? 16 : 32;   // hypothesis chunks of 32 per block (LDS ~36 KB)
  static constexpr int kFrags = TIGHT ? 2 : 1;      // B fragments (uint4) per chunk lane
  static constexpr int kBoundExp = TIGHT ? -17 : -14;
};

__device__ __forceinline__ uint32_t bf16_rne_bits(float x) {
  const uint32_t b = __float_as_uint(x);
  return (b + 0x7fffu + ((b >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_f(uint32_t u) { return __uint_as_float(u << 16); }

__device__ __forceinline__ bf16x8 frag8(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4, uint32_t a5,
                                        uint32_t a6, uint32_t a7) {
  u16x8 u;
  u[0] = (unsigned short)a0;
  u[1] = (unsigned short)a1;
  u[2] = (unsigned short)a2;
  u[3] = (unsigned short)a3;
  u[4] = (unsigned short)a4;
  u[5] = (unsigned short)a5;
  u[6] = (unsigned short)a6;
  u[7] = (unsigned short)a7;
  return __builtin_bit_cast(bf16x8, u);
}

// A fragments of point (x, y, z) for lane half h (k = 8h .. 8h + 7 of each MFMA)
template <bool TIGHT>
__device__ __forceinline__ void point_frags(float x, float y, float z, int h, bf16x8* A) {
  constexpr uint32_t one = 0x3f80;
  const uint32_t xh = bf16_rne_bits(x), yh = bf16_rne_bits(y), zh = bf16_rne_bits(z);
  const float rx = x - bf16_f(xh), ry = y - bf16_f(yh), rz = z - bf16_f(zh);  // exact
  const uint32_t xm = bf16_rne_bits(rx), ym = bf16_rne_bits(ry), zm = bf16_rne_bits(rz);
  const bool h0 = h == 0;
  static_assert(TIGHT, "the one-MFMA form was removed in round 5");
  {
    const uint32_t xl = bf16_rne_bits(rx - bf16_f(xm)), yl = bf16_rne_bits(ry - bf16_f(ym)),
                   zl = bf16_rne_bits(rz - bf16_f(zm));
    // MFMA 1  h0: xh yh zh 1 | xh yh zh 1     h1: xm ym zm 1 | xm ym zm 0
    // MFMA 2  h0: xh yh zh 0 | xl yl zl 0     h1: 0
    A[0] = h0 ? frag8(xh, yh, zh, one, xh, yh, zh, one) : frag8(xm, ym, zm, one, xm, ym, zm, 0);
    A[1] = h0 ? frag8(xh, yh, zh, 0, xl, yl, zl, 0) : frag8(0, 0, 0, 0, 0, 0, 0, 0);
  }
}

// grid: (point blocks, hypothesis groups of kChunks x 32); frag: [chunk][64
// lanes][kFrags] B fragments, hi: [chunk][32]; partial[block x][H] int32 counts.
// (a register budget of <= 256 VGPRs lets the compiler put the MFMA results
// in VGPRs, not AGPRs read back one v_accvgpr_read per element)
template <bool TIGHT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
k_plane_upper_mfma(const float* __restrict__ xyz, int64_t n, const uint4* __restrict__ frag,
                   const float* __restrict__ hi, int nch, int H, int64_t batches_per_block,
                   int32_t* __restrict__ partial) {
  using Sh = MfmaShape<TIGHT>;
  constexpr int kT = Sh::kTiles, kC = Sh::kChunks, kF = Sh::kFrags;
  __shared__ uint4 lfrag[kC * 64 * kF];
  __shared__ float lhi[kC * 32];
  __shared__ int32_t lcnt[kC * 32];
  const int c0 = blockIdx.y * kC, ncl = min(kC, nch - c0);
  for (int t = threadIdx.x; t < ncl * 64 * kF; t += kBlock) lfrag[t] = frag[(int64_t)c0 * 64 * kF + t];
  for (int t = threadIdx.x; t < ncl * 32; t += kBlock) {
    lhi[t] = hi[(int64_t)c0 * 32 + t];
    lcnt[t] = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  constexpr int kBatch = 32 * kT;
  const int64_t nbat = (n + kBatch - 1) / kBatch;
  const int64_t b0 = (int64_t)blockIdx.x * batches_per_block, b1 = min(b0 + batches_per_block, nbat);
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t b = b0 + wv; b < b1; b += kBlock / 64) {
    bf16x8 A[kT][kF];
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const int64_t i = b * kBatch + t * 32 + r;
      float x = __builtin_nanf(""), y = x, z = x;
      if (i < n) {
        const P3 v = p[i];
        x = v.x;
        y = v.y;
        z = v.z;
      }
      point_frags<TIGHT>(x, y, z, h, A[t]);
    }
    for (int c = 0; c < ncl; ++c) {
      bf16x8 B[kF];
#pragma unroll
      for (int f = 0; f < kF; ++f) B[f] = __builtin_bit_cast(bf16x8, lfrag[(c * 64 + lane) * kF + f]);
      const float hv = lhi[c * 32 + r];
      int cnt = 0;
#pragma unroll
      for (int t = 0; t < kT; ++t) {
        f32x16 d = {};
#pragma unroll
        for (int f = 0; f < kF; ++f) d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[t][f], B[f], d, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 16; ++e) cnt += fabsf(d[e]) < hv ? 1 : 0;
      }
      atomicAdd(&lcnt[c * 32 + r], cnt);  // lanes r and r + 32 hold the two row halves
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < ncl * 32; t += kBlock) {
    const int hh = c0 * 32 + t;
    if (hh < H) partial[(int64_t)blockIdx.x * H + hh] = lcnt[t];
  }
}

// ---------------------------------------------------- culled upper sweep
// Most (point, hypothesis) pairs of a RANSAC sweep are far from the plane.
// The culled sweep first puts the points in Morton order of a 2^b-per-axis
// grid over the cloud's box (two-level counting sort, below), so 64
// consecutive points — a chunk — form a compact patch.  Per chunk the wave takes the box of its
// finite points (centre c, half extents e) and tests 64 hypotheses at a time
// (lane = hypothesis):
//   |n.c + d| - (|a| ex + |b| ey + |c| ez) < limc_h
// in float32; the survivors are listed in LDS and counted 64 at a time with
// lane = hypothesis and the chunk's points broadcast (v_readlane): three fmas
// and a compare per (point, hypothesis), the float32 count |d32| < lim_h of
// k_plane_upper (lim_h >= thr + 6 2^-24 S_h + 2^-20 thr, so every float64
// inlier is counted).  Culling is conservative: for p in the box, |d_exact(p)|
// >= |dc_exact| - r_exact, the float32 dc and r are within 12.2 2^-24 S_h of
// those, and |d32(p)| < lim_h implies |d_exact(p)| < lim_h + 4 2^-24 S_h; so
// limc_h = lim_h + 20 2^-24 S_h (rounded up) never drops a pair the float32
// count would take.  The counts are the same upper bounds as k_plane_upper's
// (a pair counted here is counted there); the work is the surviving pairs.
constexpr int kCullBlock = 512;    // 8 waves (LDS ~30 KB per block, 34 KB for the exact form)
constexpr int kCullHG = 1024;      // hypotheses per block row (LDS ~29 KB)
constexpr int kCullMinN = 4096;    // smaller clouds keep the dense sweeps
constexpr int kCullCS = 128;       // points per chunk (one wave)
constexpr int kCullResident = 256 * 5;  // blocks resident at once (256 CUs x 5 by LDS)
constexpr int kCullPB = 16;        // points per batch of scalar loads

__device__ __forceinline__ uint32_t spread_bits3(uint32_t v) {  // <= 10 bits -> every third bit
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// Morton cell of a point on the 2^bits grid over mm = {min xyz, max xyz}
// (float64 on the device); clamped, non-finite coordinates land in cell 0.
struct BinGeom {
  float mn[3], sc[3], top;
};
__device__ __forceinline__ BinGeom bin_geom(const double* __restrict__ mm, int bits) {
  BinGeom g;
  const double cells = (double)(1 << bits);
  for (int a = 0; a < 3; ++a) {
    const double ext = mm[3 + a] - mm[a];
    g.mn[a] = (float)mm[a];
    g.sc[a] = ext > 0 ? (float)(cells / ext) : 0.0f;
  }
  g.top = (float)((1 << bits) - 1);
  return g;
}
__device__ __forceinline__ uint32_t bin_key(const BinGeom& g, float x, float y, float z) {
  const float v[3] = {x, y, z};
  uint32_t k = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float c = fminf(fmaxf((v[a] - g.mn[a]) * g.sc[a], 0.0f), g.top);  // NaN -> 0
    k |= spread_bits3((uint32_t)c) << a;
  }
  return k;
}

// Two-level Morton order without global atomics: the top kb bits per axis
// pick a brick (<= 512), the low lb bits a local cell (<= 512); brick-major
// then cell order is the Morton order of the full grid.  Pass 1: per-block
// brick histograms (LDS), brick-major, scanned on the device; pass 2: the
// block's points sorted by brick in an LDS stage, then written as runs (one
// run per brick and block: coalesced), the local cell in .w; pass 3: tiles
// of each brick sorted by local cell (below).  Both sorts stage the points
// themselves in LDS, so global reads and writes stay in address order.
// The order inside a cell is the LDS atomics' (the sweep does not care).
constexpr int kCBinBlock = 1024;
constexpr int kCBinPer = 4;
constexpr int kCBinChunk = kCBinBlock * kCBinPer;  // points per block and per tile (LDS stage 64 KB)
constexpr int kCBinMaxBricks = 512;
constexpr int kCBinMaxLocal = 512;

__global__ void __launch_bounds__(kCBinBlock) k_cbin_hist(const float* __restrict__ xyz, int64_t n,
                                                          const double* __restrict__ mm, int bits, int lb, int nb,
                                                          int32_t* __restrict__ bh) {
  __shared__ int32_t hist[kCBinMaxBricks];
  const BinGeom g = bin_geom(mm, bits);
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int k = threadIdx.x; k < nb; k += kCBinBlock) hist[k] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kCBinChunk;
#pragma unroll 4
  for (int j = 0; j < kCBinPer; ++j) {
    const int64_t i = base + threadIdx.x + (int64_t)j * kCBinBlock;
    if (i < n) {
      const P3 v = p[i];
      atomicAdd(&hist[bin_key(g, v.x, v.y, v.z) >> (3 * lb)], 1);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nb; k += kCBinBlock) bh[(int64_t)k * gridDim.x + blockIdx.x] = hist[k];
}

__global__ void __launch_bounds__(kCBinBlock) k_cbin_scatter(const float* __restrict__ xyz, int64_t n,
                                                             const double* __restrict__ mm, int bits, int lb, int nb,
                                                             const int32_t* __restrict__ bstart,
                                                             float4* __restrict__ tmp) {
  __shared__ float4 stage[kCBinChunk];  // the block's points sorted by brick, .w = (brick << 9) | cell
  __shared__ int32_t lstart[kCBinMaxBricks], cur[kCBinMaxBricks];
  __shared__ int32_t wsum[kCBinBlock / 64 + 1];
  const BinGeom g = bin_geom(mm, bits);
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int k = threadIdx.x; k < nb; k += kCBinBlock) cur[k] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kCBinChunk;
  const uint32_t lmask = (1u << (3 * lb)) - 1u;
  P3 v[kCBinPer];
  uint32_t code[kCBinPer];
#pragma unroll
  for (int j = 0; j < kCBinPer; ++j) {
    const int64_t i = base + threadIdx.x + (int64_t)j * kCBinBlock;
    code[j] = ~0u;
    if (i < n) {
      v[j] = p[i];
      const uint32_t key = bin_key(g, v[j].x, v[j].y, v[j].z);
      const uint32_t k = key >> (3 * lb);
      code[j] = (k << 9) | (key & lmask);
      atomicAdd(&cur[k], 1);
    }
  }
  __syncthreads();
  // exclusive scan of the block's brick counts (one brick per thread: nb <= 512 < kCBinBlock)
  const int c = threadIdx.x < nb ? cur[threadIdx.x] : 0;
  int tot;
  const int ex = block_excl_scan<kCBinBlock>(c, wsum, &tot);
  if (threadIdx.x < nb) {
    // lstart: global address of stage slot 0 for brick k (the block's run start - its stage start)
    lstart[threadIdx.x] = bstart[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] - ex;
    cur[threadIdx.x] = ex;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kCBinPer; ++j)
    if (code[j] != ~0u)
      stage[atomicAdd(&cur[code[j] >> 9], 1)] = make_float4(v[j].x, v[j].y, v[j].z, __int_as_float((int)code[j]));
  __syncthreads();
  // stage slot t of brick k -> the block's run of brick k, consecutive
  for (int t = threadIdx.x; t < tot; t += kCBinBlock) {
    const float4 e = stage[t];
    const uint32_t cd = (uint32_t)__float_as_int(e.w);
    tmp[(int64_t)lstart[cd >> 9] + t] = make_float4(e.x, e.y, e.z, __int_as_float((int)(cd & 511u)));
  }
}

// Pass 3 works on tiles: every brick's range cut into pieces of at most
// kCBinChunk points (so a tile never holds two bricks), listed by one
// workgroup; each tile is sorted by local cell in LDS on its own and written
// back in place order (coalesced).  A tile covers its whole brick, so a chunk
// of the sweep is 1 / (tile / chunk) of the brick along each axis at worst.
__global__ void __launch_bounds__(kCBinBlock) k_cbin_tiles(const int32_t* __restrict__ bstart, int nblk, int nb,
                                                           int64_t n, int2* __restrict__ tiles,
                                                           int32_t* __restrict__ ntiles) {
  __shared__ int32_t wsum[kCBinBlock / 64 + 1];
  const int k = threadIdx.x;
  int64_t s0 = 0, s1 = 0;
  if (k < nb) {
    s0 = bstart[(int64_t)k * nblk];
    s1 = k + 1 < nb ? bstart[(int64_t)(k + 1) * nblk] : n;
  }
  const int cnt = (int)((s1 - s0 + kCBinChunk - 1) / kCBinChunk);
  int tot;
  const int at = block_excl_scan<kCBinBlock>(cnt, wsum, &tot);
  for (int t = 0; t < cnt; ++t)
    tiles[at + t] = make_int2((int)(s0 + (int64_t)t * kCBinChunk), (int)min<int64_t>(s0 + (int64_t)(t + 1) * kCBinChunk, s1));
  if (threadIdx.x == 0) *ntiles = tot;
}

__global__ void __launch_bounds__(kCBinBlock) k_cbin_local(const float4* __restrict__ tmp,
                                                           const int2* __restrict__ tiles,
                                                           const int32_t* __restrict__ ntiles, int nl,
                                                           float4* __restrict__ out) {
  __shared__ float4 stage[kCBinChunk];  // the tile sorted by local cell
  __shared__ int32_t cnt[kCBinMaxLocal];
  __shared__ int32_t wsum[kCBinBlock / 64 + 1];
  if ((int)blockIdx.x >= *ntiles) return;  // block-uniform: before any barrier
  const int2 tl = tiles[blockIdx.x];
  const int s0 = tl.x, m = tl.y - tl.x;
  for (int c = threadIdx.x; c < nl; c += kCBinBlock) cnt[c] = 0;
  __syncthreads();
  float4 v[kCBinPer];
#pragma unroll
  for (int j = 0; j < kCBinPer; ++j) {
    const int t = threadIdx.x + j * kCBinBlock;
    v[j] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
    if (t < m) v[j] = tmp[s0 + t];
    if (t < m) atomicAdd(&cnt[__float_as_int(v[j].w)], 1);
  }
  __syncthreads();
  const int span = (nl + kCBinBlock - 1) / kCBinBlock;
  const int c0 = threadIdx.x * span, c1 = min(c0 + span, nl);
  int run = 0;
  for (int c = c0; c < c1; ++c) run += cnt[c];
  int tot;
  int ex = block_excl_scan<kCBinBlock>(run, wsum, &tot);
  for (int c = c0; c < c1; ++c) {
    const int u = cnt[c];
    cnt[c] = ex;
    ex += u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kCBinPer; ++j) {
    const int cl = __float_as_int(v[j].w);
    if (cl >= 0) stage[atomicAdd(&cnt[cl], 1)] = make_float4(v[j].x, v[j].y, v[j].z, 0.0f);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kCBinPer; ++j) {
    const int t = threadIdx.x + j * kCBinBlock;
    if (t < m) out[s0 + t] = stage[t];
  }
}

// all-lanes reduction of a float (EXEC full): DPP within 16-lane rows
// (l ^ 1, l ^ 2, half-row mirror, row_ror:8), then row and half swaps
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xf, 0xf, false));
}
template <class F>
__device__ __forceinline__ float wave_all_f(float v, F op) {
  v = op(v, dpp_f<0xB1>(v));
  v = op(v, dpp_f<0x4E>(v));
  v = op(v, dpp_f<0x141>(v));
  v = op(v, dpp_f<0x128>(v));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = op(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
__device__ __forceinline__ float wave_min_f(float v) {
  return wave_all_f(v, [](float a, float b) { return fminf(a, b); });
}
__device__ __forceinline__ float wave_max_f(float v) {
  return wave_all_f(v, [](float a, float b) { return fmaxf(a, b); });
}

// grid: (blocks over chunks of kCullCS points, hypothesis rows of kCullHG);
// pts: the Morton-ordered points, padded with NaN rows to a whole chunk;
// pl32 [H] float32 planes, pl64 [H] the float64 planes, lims [H] = (hi, limc,
// lo, -) (degenerate: -1, -inf, -1); partial [block x][H] int32 upper
// bounds of the counts.  Per chunk a wave takes the box of its finite points,
// tests the hypotheses 64 at a time (lane = hypothesis, coefficients from
// LDS) and lists the survivors in LDS; every 64 listed survivors (and the
// rest at the end) are counted with lane = hypothesis and the chunk's points
// read by scalar loads (wave-uniform addresses): three fmas, a compare and an
// add per (point, hypothesis), |d32| < hi.  (Round 4 measured an exact form —
// a second compare against lo and a float64 re-count of band chunks — 0.13
// ms slower than the exact round it would replace; removed in round 5.)
__global__ void __launch_bounds__(kCullBlock) k_plane_upper_cull(const float4* __restrict__ pts, int64_t n,
                                                                 const float4* __restrict__ pl32,
                                                                 const float4* __restrict__ lims, int H,
                                                                 int32_t* __restrict__ partial) {
  constexpr int kW = kCullBlock / 64, CS = kCullCS;
  __shared__ float4 lpl[kCullHG];
  __shared__ float2 llim[kCullHG];               // (hi, limc)
  __shared__ int32_t lcnt[kCullHG];
  __shared__ uint16_t lst[kW][128];
  const int h0 = blockIdx.y * kCullHG, hn = min(kCullHG, H - h0);
  for (int t = threadIdx.x; t < hn; t += kCullBlock) {
    lpl[t] = pl32[h0 + t];
    const float4 l = lims[h0 + t];
    llim[t] = make_float2(l.x, l.y);
    lcnt[t] = 0;
  }
  __syncthreads();
  // the wave index as a scalar: chunk addresses are wave-uniform (scalar loads)
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t below = (1ull << lane) - 1ull;
  const int64_t nchunk = (n + CS - 1) / CS;
  const int64_t cstep = (int64_t)gridDim.x * kW;
  float4 nxt[CS / 64];  // the next chunk's points, loaded while this one is swept
  {
    const int64_t c0 = min<int64_t>((int64_t)blockIdx.x * kW + wv, nchunk - 1);
#pragma unroll
    for (int j = 0; j < CS / 64; ++j) nxt[j] = pts[c0 * CS + j * 64 + lane];
  }
  for (int64_t c = (int64_t)blockIdx.x * kW + wv; c < nchunk; c += cstep) {
    const float4* cp = pts + c * CS;  // wave-uniform
    float4 cur[CS / 64];
#pragma unroll
    for (int j = 0; j < CS / 64; ++j) cur[j] = nxt[j];
    {
      const int64_t cn = min(c + cstep, nchunk - 1);
#pragma unroll
      for (int j = 0; j < CS / 64; ++j) nxt[j] = pts[cn * CS + j * 64 + lane];
    }
    float mnx = INFINITY, mny = INFINITY, mnz = INFINITY, mxx = -INFINITY, mxy = -INFINITY, mxz = -INFINITY;
#pragma unroll
    for (int j = 0; j < CS / 64; ++j) {
      const float4 v = cur[j];
      const bool fin = __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z);
      mnx = fminf(mnx, fin ? v.x : INFINITY);
      mny = fminf(mny, fin ? v.y : INFINITY);
      mnz = fminf(mnz, fin ? v.z : INFINITY);
      mxx = fmaxf(mxx, fin ? v.x : -INFINITY);
      mxy = fmaxf(mxy, fin ? v.y : -INFINITY);
      mxz = fmaxf(mxz, fin ? v.z : -INFINITY);
    }
    auto u = [](float f) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(f))); };
    mnx = u(wave_min_f(mnx));
    mny = u(wave_min_f(mny));
    mnz = u(wave_min_f(mnz));
    mxx = u(wave_max_f(mxx));
    mxy = u(wave_max_f(mxy));
    mxz = u(wave_max_f(mxz));
    if (!(mnx <= mxx)) continue;  // no finite point: nothing to count
    const float cx = 0.5f * mnx + 0.5f * mxx, cy = 0.5f * mny + 0.5f * mxy, cz = 0.5f * mnz + 0.5f * mxz;
    const float ex = 0.5f * mxx - 0.5f * mnx, ey = 0.5f * mxy - 0.5f * mny, ez = 0.5f * mxz - 0.5f * mnz;
    // count the listed hypotheses [0, g) against the chunk's points
    auto eval = [&](int g) {
      const bool act = lane < g;
      const int h = act ? (int)lst[wv][lane] : 0;
      const float4 p = lpl[h];
      const float hi = act ? llim[h].x : -1.0f;
      int chi = 0;  // |d32| < hi
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
      for (int k0 = 0; k0 < CS; k0 += kCullPB) {
        float4 q[kCullPB];
#pragma unroll
        for (int j = 0; j < kCullPB; ++j) q[j] = cp[k0 + j];  // scalar loads
#pragma unroll
        for (int j = 0; j < kCullPB; ++j) {
          const float ad = fabsf(fmaf(p.x, q[j].x, fmaf(p.y, q[j].y, fmaf(p.z, q[j].z, p.w))));
          chi += ad < hi ? 1 : 0;
        }
      }
      if (act && chi) atomicAdd(&lcnt[h], chi);
    };
    int nl = 0;  // wave-uniform list length (< 64 between groups)
    for (int g0 = 0; g0 < hn; g0 += 64) {
      const int h = g0 + lane;
      bool surv = false;
      if (h < hn) {
        const float4 p = lpl[h];
        const float dc = fmaf(p.x, cx, fmaf(p.y, cy, fmaf(p.z, cz, p.w)));
        const float r = fmaf(fabsf(p.x), ex, fmaf(fabsf(p.y), ey, fabsf(p.z) * ez));
        surv = fabsf(dc) - r < llim[h].y;
      }
      const uint64_t m = __ballot(surv);
      if (surv) lst[wv][nl + __popcll(m & below)] = (uint16_t)h;
      nl += __popcll(m);
      __builtin_amdgcn_wave_barrier();
      if (nl >= 64) {
        eval(64);
        const int rest = nl - 64;
        const uint16_t mv = lane < rest ? lst[wv][64 + lane] : 0;
        __builtin_amdgcn_wave_barrier();
        if (lane < rest) lst[wv][lane] = mv;
        __builtin_amdgcn_wave_barrier();
        nl = rest;
      }
    }
    if (nl > 0) eval(nl);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  for (int t = threadIdx.x; t < hn; t += kCullBlock) partial[(int64_t)blockIdx.x * H + h0 + t] = lcnt[t];
}

// Host side of the fragments: bf16 (round to nearest even) of a float
static uint16_t bf16_rne_host(float x) {
  uint32_t b;
  std::memcpy(&b, &x, 4);
  return (uint16_t)((b + 0x7fffu + ((b >> 16) & 1u)) >> 16);
}
static float bf16_value(uint16_t u) {
  const uint32_t b = (uint32_t)u << 16;
  float f;
  std::memcpy(&f, &b, 4);
  return f;
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

__global__ void k_mark_degenerate(const uint8_t* __restrict__ degenerate, int H, int64_t* __restrict__ counts) {
  int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h < H && degenerate[h] == 1) counts[h] = -1;
}

constexpr int kSumBlocksX = 64;

// Sigma |d| over the points with |d| < thr, one hypothesis per blockIdx.y, as
// an exact fx sum (common.hpp; |d| < thr bounds every term): the same bits for
// any split of the cloud over blocks or ranks.  partial: [y][x] {lo, hi}.
template <class T>
__global__ void __launch_bounds__(kBlock) k_plane_abs_sum(const T* __restrict__ xyz, int64_t n,
                                                          const double* __restrict__ pl64, double thr, double scale,
                                                          int64_t* __restrict__ partial) {
  __shared__ int64_t sh[(kBlock / 64) * 2];
  const double* pl = pl64 + 4 * blockIdx.y;
  int64_t acc[1] = {0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double x, y, z;
    load3(xyz, i, x, y, z);
    double d = plane_dist64(pl, x, y, z);
    if (d < thr) acc[0] += fx_term(d, scale);
  }
  block_fx<kBlock, 1>(acc, sh, partial + 2 * ((int64_t)blockIdx.y * gridDim.x + blockIdx.x));
}

static int abs_sum_blocks(int64_t n) {
  return (int)std::max<int64_t>(kSumBlocksX, (n + (int64_t)kBlock * kFxLaneTerms - 1) / ((int64_t)kBlock * kFxLaneTerms));
}

template <class T>
__global__ void __launch_bounds__(kBlock) k_plane_flags(const T* __restrict__ xyz, int64_t n, double a, double b,
                                                        double c, double d, double thr, uint8_t* __restrict__ flags) {
  const double pl[4] = {a, b, c, d};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double x, y, z;
    load3(xyz, i, x, y, z);
    flags[i] = plane_dist64(pl, x, y, z) < thr ? 1 : 0;
  }
}

// Plane selection of the reference's PointCloudSelections (PointCloud.py:
// 278-290, 400-404): s = ((x*a + y*b) + z*c + d) / nrm, unfused, the order of
// numpy's `(p*abc).sum(1) + d` (distance2plane); flag = |s| < thr (BAND 0) or
// lo < s < hi (BAND 1), xor invert.  dist (optional) receives s.
template <bool BAND, class T>
__global__ void __launch_bounds__(kBlock) k_plane_band(const T* __restrict__ xyz, int64_t n, double a, double b,
                                                       double c, double d, double nrm, double lo, double hi,
                                                       int invert, uint8_t* __restrict__ flags,
                                                       double* __restrict__ dist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x = (double)xyz[3 * i], y = (double)xyz[3 * i + 1], z = (double)xyz[3 * i + 2];
    const double t = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(x, a), __dmul_rn(y, b)), __dmul_rn(z, c)), d);
    const double s = __ddiv_rn(t, nrm);
    if (dist) dist[i] = s;
    if (flags) {
      const bool in = BAND ? (s > lo && s < hi) : (fabs(s) < hi);
      flags[i] = (uint8_t)(in != (invert != 0));
    }
  }
}

constexpr int kMomBlocks = 2048;  // gathers over the inlier list: enough waves in flight

// GetPlaneFromPoints moments over the inliers as exact fx sums (common.hpp),
// so the refit plane is the same bits for any split of the inliers over
// blocks or ranks.  pass 1 (pass2 == 0): {x, y, z}; pass 2: centred
// {xx, xy, xz, yy, yz, zz}.  sc: the fx scales of the pass's sums.
struct MomScales {
  double s[6];
};

template <class T>
__global__ void __launch_bounds__(kBlock) k_plane_moments(const T* __restrict__ xyz, const int32_t* __restrict__ idx,
                                                          int64_t m, double cx, double cy, double cz, int pass2,
                                                          MomScales sc, int64_t* __restrict__ partial) {
  __shared__ int64_t sh[(kBlock / 64) * 12];
  int64_t acc[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    int64_t i = idx ? idx[j] : j;
    double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (!pass2) {
      acc[0] += fx_term(x, sc.s[0]);
      acc[1] += fx_term(y, sc.s[1]);
      acc[2] += fx_term(z, sc.s[2]);
    } else {
      double r0 = x - cx, r1 = y - cy, r2 = z - cz;
      acc[0] += fx_term(r0 * r0, sc.s[0]);
      acc[1] += fx_term(r0 * r1, sc.s[1]);
      acc[2] += fx_term(r0 * r2, sc.s[2]);
      acc[3] += fx_term(r1 * r1, sc.s[3]);
      acc[4] += fx_term(r1 * r2, sc.s[4]);
      acc[5] += fx_term(r2 * r2, sc.s[5]);
    }
  }
  block_fx<kBlock, 6>(acc, sh, partial + (int64_t)blockIdx.x * 12);
}

// segment_plane's last step in one read of the cloud: the inlier flags of the
// best plane and the first moments pass (fx sums of x, y, z over the inliers)
template <class T>
__global__ void __launch_bounds__(kBlock) k_plane_flags_sum(const T* __restrict__ xyz, int64_t n, double a,
                                                            double b, double c, double d, double thr, MomScales sc,
                                                            uint8_t* __restrict__ flags,
                                                            int64_t* __restrict__ partial) {
  __shared__ int64_t sh[(kBlock / 64) * 6];
  const double pl[4] = {a, b, c, d};
  int64_t acc[3] = {0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double x, y, z;
    load3(xyz, i, x, y, z);
    const bool in = plane_dist64(pl, x, y, z) < thr;
    flags[i] = in ? 1 : 0;
    if (in) {
      acc[0] += fx_term(x, sc.s[0]);
      acc[1] += fx_term(y, sc.s[1]);
      acc[2] += fx_term(z, sc.s[2]);
    }
  }
  block_fx<kBlock, 3>(acc, sh, partial + (int64_t)blockIdx.x * 6);
}

// Second moments pass with the centroid formed on the device: c = (fx sum of
// the first pass) / k, the value the host forms (fx_value = fx_to_double);
// k = *count (the compaction's), the first pass's digit sums in s1 (3 rows).
template <class T>
__global__ void __launch_bounds__(kBlock) k_plane_moments_c(const T* __restrict__ xyz,
                                                            const int32_t* __restrict__ idx,
                                                            const int64_t* __restrict__ count,
                                                            const int64_t* __restrict__ s1, int q0, int q1, int q2,
                                                            MomScales sc, int64_t* __restrict__ partial) {
  __shared__ int64_t sh[(kBlock / 64) * 12];
  const int64_t m = *count;
  const double k = (double)m;
  const double cx = fx_value(s1[0], s1[1], q0) / k, cy = fx_value(s1[2], s1[3], q1) / k,
               cz = fx_value(s1[4], s1[5], q2) / k;
  int64_t acc[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx[j];
    const double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    const double r0 = x - cx, r1 = y - cy, r2 = z - cz;
    acc[0] += fx_term(r0 * r0, sc.s[0]);
    acc[1] += fx_term(r0 * r1, sc.s[1]);
    acc[2] += fx_term(r0 * r2, sc.s[2]);
    acc[3] += fx_term(r1 * r1, sc.s[3]);
    acc[4] += fx_term(r1 * r2, sc.s[4]);
    acc[5] += fx_term(r2 * r2, sc.s[5]);
  }
  block_fx<kBlock, 6>(acc, sh, partial + (int64_t)blockIdx.x * 12);
}

static int mom_blocks(int64_t m) {
  const int64_t need = (m + (int64_t)kBlock * kFxLaneTerms - 1) / ((int64_t)kBlock * kFxLaneTerms);
  return (int)std::max<int64_t>(1, std::max<int64_t>(need, std::min<int64_t>(kMomBlocks, (m + kBlock - 1) / kBlock)));
}

// fx exponents of the moment sums from A = the largest |coordinate| of the
// cloud (every rank of a sharded cloud passes the global one): |x| <= A;
// centred |x - c| <= 2A, products <= 4A^2 (x 1.01 for rounding)
static void mom_fx_exps(double A, bool pass2, int q[6]) {
  for (int k = 0; k < 6; ++k) q[k] = pass2 ? fx_exp(4.0 * A * A * 1.01) : (k < 3 ? fx_exp(A) : 0);
}

// The second pass's exponents from the cloud's extent E (largest max - min):
// the inliers and their centroid lie in the bounding box, so |x - c| <= E
// (x 1.01 for rounding).  At a georeferenced offset (|x| ~ 5e5, E ~ 50) the
// |x| bound would coarsen the centred products' quantum by 2^30.
static void mom_fx_exps_span(double E, int q[6]) {
  for (int k = 0; k < 6; ++k) q[k] = fx_exp(E * E * 1.03);
}

template <class T>
__global__ void k_gather_samples(const T* __restrict__ xyz, const int32_t* __restrict__ idx, int64_t m,
                                 T* __restrict__ out) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  int64_t i = idx[j];
  out[3 * j] = xyz[3 * i];
  out[3 * j + 1] = xyz[3 * i + 1];
  out[3 * j + 2] = xyz[3 * i + 2];
}

// ------------------------------------------- plane math (host and device)
// One definition for both sides: segment_plane's culled path forms the
// hypotheses on the device (k_ransac_setup), the other paths on the host;
// compiled with -ffp-contract=off and correctly rounded sqrt / division on
// both, the planes are the same bits.
#define O3DX_HD __host__ __device__
O3DX_HD inline void hcross(const double u[3], const double v[3], double o[3]) {
  o[0] = u[1] * v[2] - u[2] * v[1];
  o[1] = u[2] * v[0] - u[0] * v[2];
  o[2] = u[0] * v[1] - u[1] * v[0];
}
O3DX_HD inline double hdot(const double u[3], const double v[3]) { return (u[0] * v[0] + u[1] * v[1]) + u[2] * v[2]; }

O3DX_HD inline void plane_from_centred(const double c[3], const double mo[6], double pl[4]) {
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
  double norm = sqrt(hdot(abc, abc));
  if (norm == 0) {
    pl[0] = pl[1] = pl[2] = pl[3] = 0;
    return;
  }
  for (int a = 0; a < 3; ++a) abc[a] /= norm;
  pl[0] = abc[0]; pl[1] = abc[1]; pl[2] = abc[2];
  pl[3] = -hdot(abc, c);
}

// ComputeTrianglePlane (k == 3) / GetPlaneFromPoints (k > 3), float64
O3DX_HD inline void plane_from_pts(const double* P, int k, double pl[4]) {
  if (k == 3) {
    double e0[3] = {P[3] - P[0], P[4] - P[1], P[5] - P[2]};
    double e1[3] = {P[6] - P[0], P[7] - P[1], P[8] - P[2]};
    double abc[3];
    hcross(e0, e1, abc);
    double norm = sqrt(hdot(abc, abc));
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

// 1: degenerate (count -1); 2: non-finite coefficients (count 0); 0: a plane
O3DX_HD inline int plane_kind(const double* pl) {
  if (pl[0] == 0 && pl[1] == 0 && pl[2] == 0 && pl[3] == 0) return 1;
  for (int a = 0; a < 4; ++a)
    if (!(pl[a] == pl[a] && pl[a] <= DBL_MAX && pl[a] >= -DBL_MAX)) return 2;
  return 0;
}

// The culled sweep's per-hypothesis limits (hi, limc, lo, 0), §4.3:
// S = |a| max|x| + |b| max|y| + |c| max|z| + |d|, g = 6 2^-24 S + 2^-20 thr,
// hi = thr + g and limc = hi + 20 2^-24 S rounded up, lo = thr - g rounded
// down (0 when thr <= g); degenerate: never counted.
O3DX_HD inline float f32_up(double v) {
  float f = (float)v;
  return (double)f < v ? nextafterf(f, INFINITY) : f;
}
O3DX_HD inline float f32_down(double v) {
  float f = (float)v;
  return (double)f > v ? nextafterf(f, -INFINITY) : f;
}
O3DX_HD inline float4 cull_limits(const double* pl, const double absmax[3], double thr, int kind) {
  if (kind == 1) return make_float4(-1.0f, -INFINITY, -1.0f, 0.f);
  const double S = fabs(pl[0]) * absmax[0] + fabs(pl[1]) * absmax[1] + fabs(pl[2]) * absmax[2] + fabs(pl[3]);
  const double g = 6.0 * 5.9604644775390625e-08 * S + 9.5367431640625e-07 * thr;
  const float lim = f32_up(thr + g);
  const float lo = thr - g > 0 ? f32_down(thr - g) : 0.0f;
  return make_float4(lim, f32_up((double)lim + 20.0 * 5.9604644775390625e-08 * S), lo, 0.f);
}

// segment_plane's culled path forms the hypotheses on the device: per
// hypothesis plane_from_pts over its gathered sample coordinates, the float32
// plane, the culled sweep's limits from the device bounds, and the float64
// plane (+ the bounds, thread 0) into the read-back block.
__global__ void __launch_bounds__(kBlock) k_ransac_setup(const float* __restrict__ scoord, int H, int rn,
                                                         const double* __restrict__ mm, double thr,
                                                         float4* __restrict__ pl32, float4* __restrict__ lims,
                                                         uint8_t* __restrict__ degen, double* __restrict__ pl64_out,
                                                         double* __restrict__ mm_out) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h == 0)
    for (int a = 0; a < 6; ++a) mm_out[a] = mm[a];
  if (h >= H) return;
  double absmax[3];
  for (int a = 0; a < 3; ++a) absmax[a] = fmax(fabs(mm[a]), fabs(mm[3 + a]));
  double P[48];
  for (int j = 0; j < rn * 3; ++j) P[j] = (double)scoord[(int64_t)h * rn * 3 + j];
  double pl[4];
  plane_from_pts(P, rn, pl);
  const int kind = plane_kind(pl);
  for (int a = 0; a < 4; ++a) pl64_out[4 * (int64_t)h + a] = pl[a];
  pl32[h] = make_float4((float)pl[0], (float)pl[1], (float)pl[2], (float)pl[3]);
  lims[h] = cull_limits(pl, absmax, thr, kind);
  degen[h] = (uint8_t)kind;
}

static bool plane_is_zero(const double* pl) { return pl[0] == 0 && pl[1] == 0 && pl[2] == 0 && pl[3] == 0; }

// ------------------------------------------------------------ workspaces

// count geometry: nwp ranges of bpw batches of `batch` points
// count geometry: nwp ranges of bpw batches of `batch` points.  Few
// hypothesis chunks (a re-count of a handful of hypotheses) get more ranges,
// so the launch still fills the chip (~16K waves), within the partial
// buffer's capacity (cap_ints >= nwp * H).
static void count_geometry(int64_t n, int batch, int* nwp, int64_t* bpw, int nchunks = 32, int H = 1,
                           size_t cap_ints = 0) {
  const int64_t nb = std::max<int64_t>(1, (n + batch - 1) / batch);
  int64_t want = std::max<int64_t>(kCountWaves, 16384 / std::max(nchunks, 1));
  if (cap_ints) want = std::min<int64_t>(want, std::max<int64_t>(kCountWaves, (int64_t)(cap_ints / std::max(H, 1))));
  *nwp = (int)std::min<int64_t>(want, nb);
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
  uint4* mfrag;  // k_plane_upper_mfma: B fragments [chunk][64], then hi [chunk][32] (same upload)
  float* mhi;
  int32_t* partial;
  size_t partial_ints;
  uint32_t* flags;  // (batch, hypothesis chunk) window bitmap of the brute-force count
  int64_t* counts;
  int64_t* sum_partial;
  // culled sweep: Morton-ordered copy of the points and its counting sort
  float4* sorted;
  float4* tmp;
  int2* tiles;
  int32_t* ntiles;
  int32_t* bh;
  int32_t* bstart;
  int32_t* bscan;
  int bits;
  bool binned;        // sorted holds this call's points
};

// grid bits per axis of the culled sweep's Morton order: ~8 points per cell
static int cull_bits(int64_t n) {
  const double b = std::log2(std::max<double>((double)n, 8.0) / 8.0) / 3.0;
  return std::max(1, std::min(6, (int)std::lround(b)));  // <= 3 + 3: the stage entry's fields
}

static size_t count_carve(Arena& ar, int64_t n, int H, CountWs* w) {
  H = std::max(H, 1);
  // the per-hypothesis inputs in one block: one upload (upload_planes)
  const size_t nch = ((size_t)H + 31) / 32, omf = (65 * (size_t)H + 15) & ~(size_t)15;
  uint8_t* up = ar.take<uint8_t>(omf + nch * (64 * 32 + 32 * 4));
  w->pl32 = reinterpret_cast<float4*>(up);
  w->band = reinterpret_cast<float4*>(up + 16 * (size_t)H);
  w->pl64 = reinterpret_cast<double*>(up + 32 * (size_t)H);
  w->degen = up + 64 * (size_t)H;
  w->mfrag = reinterpret_cast<uint4*>(up + omf);
  w->mhi = reinterpret_cast<float*>(up + omf + nch * 64 * 32);
  w->partial_ints = (size_t)std::max(count_blocks(n), kCountWaves) * H;
  w->partial = ar.take<int32_t>(w->partial_ints);
  w->flags = ar.take<uint32_t>((size_t)count_flag_words(n, H, kMinBatchPts, kMinHC));
  w->counts = ar.take<int64_t>(H);
  w->sum_partial = ar.take<int64_t>((size_t)2 * abs_sum_blocks(n) * H);
  w->bits = cull_bits(n);
  const int64_t nbh = (int64_t)kCBinMaxBricks * ((n + kCBinChunk - 1) / kCBinChunk);
  w->sorted = ar.take<float4>((size_t)n + kCullCS);  // + NaN rows to a whole chunk
  w->tmp = ar.take<float4>((size_t)n);
  w->tiles = ar.take<int2>((size_t)(n + kCBinChunk - 1) / kCBinChunk + kCBinMaxBricks);
  w->ntiles = ar.take<int32_t>(4);
  w->bh = ar.take<int32_t>((size_t)nbh + 1);
  w->bstart = ar.take<int32_t>((size_t)nbh + 1);
  w->bscan = ar.take<int32_t>(scan_workspace_ints(nbh + 1));
  w->binned = false;
  return ar.used;
}

// scale of |a x| + |b y| + |c z| + |d| over the cloud, for the float32 band
static void upload_planes(const double* planes, int H, const double absmax[3], double thr, CountWs& w,
                          std::vector<float4>& p32, std::vector<float4>& bnd, std::vector<uint8_t>& dg,
                          std::vector<uint8_t>& st, hipStream_t s, int* rc, double* hi_max = nullptr,
                          int mfma = 0) {  // 1 / 2: k_plane_upper_mfma<false / true>'s operands
  if (hi_max) *hi_max = -1.0;
  const bool band_off = getenv("O3DX_RANSAC_BAND_OFF") != nullptr;
  p32.resize(H);
  bnd.resize(H);
  dg.resize(H);
  for (int h = 0; h < H; ++h) {
    const double* pl = planes + 4 * h;
    // 1: degenerate (count -1); 2: non-finite coefficients (count 0: no
    // distance is < thr)
    dg[h] = plane_is_zero(pl) ? 1
            : (std::isfinite(pl[0]) && std::isfinite(pl[1]) && std::isfinite(pl[2]) && std::isfinite(pl[3])) ? 0
                                                                                                            : 2;
    p32[h] = make_float4((float)pl[0], (float)pl[1], (float)pl[2], (float)pl[3]);
    double S = std::fabs(pl[0]) * absmax[0] + std::fabs(pl[1]) * absmax[1] + std::fabs(pl[2]) * absmax[2] +
               std::fabs(pl[3]);
    // float32 error of the fma chain: the four coefficients rounded (2^-24 S)
    // + three fma roundings (each <= 2^-24 S); 6 for margin, + 2^-20 thr for
    // the float32 rounding of lo / hi and Open3D's own float64 rounding
    double g = 6.0 * std::ldexp(1.0, -24) * S + std::ldexp(1.0, -20) * thr;
    float lo = (float)(thr - g), hi = (float)(thr + g);
    if (hi_max && !dg[h]) *hi_max = std::max(*hi_max, thr + g);
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
    if (mfma == 3) bnd[h] = cull_limits(pl, absmax, thr, dg[h]);  // k_plane_upper_cull (as k_ransac_setup)
  }
  *rc = 0;
  // one copy of the block laid out as count_carve placed it
  uint8_t* base = reinterpret_cast<uint8_t*>(w.pl32);
  const size_t ob = reinterpret_cast<uint8_t*>(w.band) - base, o64 = reinterpret_cast<uint8_t*>(w.pl64) - base,
               odg = w.degen - base;
  const size_t nch = ((size_t)H + 31) / 32, omf = reinterpret_cast<uint8_t*>(w.mfrag) - base,
               ohi = reinterpret_cast<uint8_t*>(w.mhi) - base;
  const bool frags = mfma == 2;
  st.assign(frags ? ohi + nch * 32 * 4 : odg + H, 0);  // the caller keeps it alive until the stream is synchronised
  std::memcpy(st.data(), p32.data(), H * sizeof(float4));
  std::memcpy(st.data() + ob, bnd.data(), H * sizeof(float4));
  std::memcpy(st.data() + o64, planes, 4 * H * sizeof(double));
  std::memcpy(st.data() + odg, dg.data(), H);
  if (frags) {
    // k_plane_upper_mfma's B operand: hypothesis j is column j % 32 of chunk
    // j / 32; bf16 parts (round to nearest) of the float64 plane.  MFMA 1 lane
    // r (ah bh ch dh | am bm cm dm), lane r + 32 (ah bh ch dl | am bm cm 0);
    // MFMA 2 lane r (al bl cl 0 | ah bh ch 0), lane r + 32 zero.  ("m" is the
    // second part, "l" the third.)
    const int nf = 2;
    uint16_t* fr = reinterpret_cast<uint16_t*>(st.data() + omf);
    float* hv = reinterpret_cast<float*>(st.data() + ohi);
    for (size_t j = 0; j < nch * 32; ++j) hv[j] = -1.0f;
    for (int j = 0; j < H; ++j) {
      if (dg[j]) continue;  // zero fragments, hi -1: never counted
      const double* pl = planes + 4 * j;
      uint16_t P[3][4];  // parts: h, m, l
      for (int a = 0; a < 4; ++a) {
        double rem = pl[a];
        for (int k = 0; k < 3; ++k) {
          P[k][a] = bf16_rne_host((float)rem);
          rem -= (double)bf16_value(P[k][a]);
        }
      }
      const uint16_t(&h_)[4] = P[0];
      const uint16_t(&m_)[4] = P[1];
      const uint16_t(&l_)[4] = P[2];
      auto put = [&](int lane, int f, const uint16_t (&v)[8]) {
        std::memcpy(fr + (((size_t)(j / 32) * 64 + lane) * nf + f) * 8, v, 16);
      };
      const int r = j % 32;
      put(r, 0, {h_[0], h_[1], h_[2], h_[3], m_[0], m_[1], m_[2], m_[3]});
      put(r + 32, 0, {h_[0], h_[1], h_[2], l_[3], m_[0], m_[1], m_[2], 0});
      put(r, 1, {l_[0], l_[1], l_[2], 0, h_[0], h_[1], h_[2], 0});
      put(r + 32, 1, {0, 0, 0, 0, 0, 0, 0, 0});
      const double S = std::fabs(pl[0]) * absmax[0] + std::fabs(pl[1]) * absmax[1] + std::fabs(pl[2]) * absmax[2] +
                       std::fabs(pl[3]);
      // O3DX_RANSAC_BAND_OFF (test hook, tests/test_gpu_kernels.py): count
      // |d_mfma| < thr itself, so a test can bound the sweep's own error
      const double band = band_off ? 0.0 : std::ldexp(1.0, MfmaShape<true>::kBoundExp) * S;
      const double lim = thr + band + 1e-30;
      float f = (float)lim;
      if ((double)f < lim) f = std::nextafter(f, INFINITY);
      hv[(j / 32) * 32 + r] = f;
    }
  }
  // through a pinned staging buffer (a direct DMA; a pageable source takes
  // the runtime's staged, blocking path).  An event recorded behind each copy
  // out of it is waited on before the buffer is written again (a caller that
  // returned early on an error may have left that copy in flight).
  constexpr size_t kPinCap = 1 << 20;
  static thread_local void* pin = nullptr;
  static thread_local hipEvent_t pin_done = nullptr;
  if (st.size() <= kPinCap && !pin && hipHostMalloc(&pin, kPinCap, hipHostMallocDefault) != hipSuccess) pin = nullptr;
  if (pin && !pin_done && hipEventCreateWithFlags(&pin_done, hipEventDisableTiming) != hipSuccess) pin_done = nullptr;
  const void* src = st.data();
  const bool staged = pin && pin_done && st.size() <= kPinCap;
  if (staged) {
    if (hipEventSynchronize(pin_done) != hipSuccess) {
      *rc = fail(O3DX_EIO, "plane upload: staging buffer wait failed");
      return;
    }
    std::memcpy(pin, st.data(), st.size());
    src = pin;
  }
  if (hipMemcpyAsync(base, src, st.size(), hipMemcpyHostToDevice, s) != hipSuccess)
    *rc = fail(O3DX_EIO, "plane upload failed");
  else if (staged && hipEventRecord(pin_done, s) != hipSuccess)
    *rc = fail(O3DX_EIO, "plane upload: event record failed");
}

static int absmax_of(const float* xyz, int64_t n, void* aabb_ws, double* mm_dev, hipStream_t s, double out[3]) {
  double mm[6];
  O3DX_TRY(aabb_device(xyz, n, mm_dev, aabb_ws, s));
  O3DX_TRY(read_back(mm, mm_dev, 6 * sizeof(double), s));
  for (int a = 0; a < 3; ++a) out[a] = std::max(std::fabs(mm[a]), std::fabs(mm[3 + a]));
  return 0;
}

static int run_count(const float* xyz, int64_t n, const double* planes, int H, double thr, CountWs& w, void* aabb_ws,
                     double* mm_dev, hipStream_t s, std::vector<int64_t>& counts, const double* absmax_in = nullptr) {
  double absmax[3];
  if (absmax_in) std::memcpy(absmax, absmax_in, sizeof(absmax));
  else O3DX_TRY(absmax_of(xyz, n, aabb_ws, mm_dev, s, absmax));
  std::vector<float4> p32;
  std::vector<float4> bnd;
  std::vector<uint8_t> dg;
  std::vector<uint8_t> st;
  int rc;
  upload_planes(planes, H, absmax, thr, w, p32, bnd, dg, st, s, &rc);
  if (rc) return rc;
  KTimer kt("plane_count", s);
  {
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
    // the default: every point against every hypothesis on the VALU
    // measured: 6 waves/SIMD fastest (r03); re-counts of a few hypotheses
    // (segment_plane's exact rounds) take a narrower chunk
    const int hc = H <= 8 ? 8 : H <= 16 ? 16 : 32, pl = 16;
    int nwp;
    int64_t bpw;
    const int nchunks = (H + hc - 1) / hc;
    count_geometry(n, 64 * pl, &nwp, &bpw, nchunks, H, w.partial_ints);
    const int ncg = (nchunks + kBlock / 64 - 1) / (kBlock / 64);  // blocks per batch range
    const int64_t nwords = count_flag_words(n, H, 64 * pl, hc);
    const unsigned fgrid = grid_for(nwords, kBlock / 64, 16384);
    auto kcount = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)(nwp * ncg)), dim3(kBlock), 0, s, xyz, n, w.pl32, H, Llo, wbits, bpw,
                         nwp, ncg, w.partial, w.flags);
    };
    if (hc == 32) kcount(k_plane_count_w6<32, 16, 0>);
    else if (hc == 16) kcount(k_plane_count_w8<16, 16, 0>);
    else kcount(k_plane_count_w8<8, 16, 0>);
    O3DX_TRY(reduce_columns_i32_to_i64(w.partial, nwp, H, w.counts, s));
    if (hc == 32)
      hipLaunchKernelGGL((k_plane_fixup<32, 16>), dim3(fgrid), dim3(kBlock), 0, s, xyz, n, w.pl32, w.pl64, H, thr,
                         Llo, wbits, w.flags, nwords, w.counts);
    else if (hc == 16)
      hipLaunchKernelGGL((k_plane_fixup<16, 16>), dim3(fgrid), dim3(kBlock), 0, s, xyz, n, w.pl32, w.pl64, H, thr,
                         Llo, wbits, w.flags, nwords, w.counts);
    else
      hipLaunchKernelGGL((k_plane_fixup<8, 16>), dim3(fgrid), dim3(kBlock), 0, s, xyz, n, w.pl32, w.pl64, H, thr,
                         Llo, wbits, w.flags, nwords, w.counts);
  }
  hipLaunchKernelGGL(k_mark_degenerate, dim3((H + 255) / 256), dim3(256), 0, s, w.degen, H, w.counts);
  kt.stop();
  counts.resize(H);
  O3DX_TRY(read_back(counts.data(), w.counts, H * sizeof(int64_t), s));
  O3DX_HIP(hipGetLastError());
  return 0;
}

// Morton order of the points for the culled sweep; mm_dev: the cloud's
// min / max on the device (no host wait)
static int bin_points(const float* xyz, int64_t n, const double* mm_dev, CountWs& w, hipStream_t s) {
  const int kb = std::min(3, w.bits), lb = w.bits - kb, nb = 1 << (3 * kb), nl = 1 << (3 * lb);
  const int nblk = (int)((n + kCBinChunk - 1) / kCBinChunk);
  KTimer kt("plane_bin", s);
  hipLaunchKernelGGL(k_cbin_hist, dim3(nblk), dim3(kCBinBlock), 0, s, xyz, n, mm_dev, w.bits, lb, nb, w.bh);
  O3DX_TRY(exclusive_scan_i32(w.bh, w.bstart, (int64_t)nb * nblk, w.bscan, s));
  hipLaunchKernelGGL(k_cbin_scatter, dim3(nblk), dim3(kCBinBlock), 0, s, xyz, n, mm_dev, w.bits, lb, nb, w.bstart,
                     w.tmp);
  hipLaunchKernelGGL(k_cbin_tiles, dim3(1), dim3(kCBinBlock), 0, s, w.bstart, nblk, nb, n, w.tiles, w.ntiles);
  hipLaunchKernelGGL(k_cbin_local, dim3(nblk + nb), dim3(kCBinBlock), 0, s, w.tmp, w.tiles, w.ntiles, nl, w.sorted);
  O3DX_HIP(hipMemsetAsync(w.sorted + n, 0xff, kCullCS * sizeof(float4), s));  // NaN rows
  O3DX_HIP(hipGetLastError());
  w.binned = true;
  return 0;
}

// The culled sweep over w.sorted with the limits already in w.pl32 / w.band /
// w.degen (host upload or k_ransac_setup): per-hypothesis counts (degenerate
// -1) into counts_dev, no host wait.
static int launch_cull(int64_t n, int H, CountWs& w, hipStream_t s, int64_t* counts_dev) {
  const int64_t nchunk = (n + kCullCS - 1) / kCullCS;
  const int64_t rows = std::max<int64_t>(1, std::min<int64_t>((int64_t)(w.partial_ints / std::max(H, 1)), 2048));
  // one resident wave per chunk stream: 5 blocks per CU (LDS ~30 KB each)
  const int64_t per_block = kCullBlock / 64;
  const unsigned gx = (unsigned)std::min<int64_t>(std::min<int64_t>(rows, kCullResident),
                                                  (nchunk + per_block - 1) / per_block);
  const unsigned gy = (unsigned)((H + kCullHG - 1) / kCullHG);
  hipLaunchKernelGGL(k_plane_upper_cull, dim3(gx, gy), dim3(kCullBlock), 0, s, w.sorted, n, w.pl32, w.band, H,
                     w.partial);
  O3DX_TRY(reduce_columns_i32_to_i64(w.partial, gx, H, counts_dev, s));
  hipLaunchKernelGGL(k_mark_degenerate, dim3((H + 255) / 256), dim3(256), 0, s, w.degen, H, counts_dev);
  O3DX_HIP(hipGetLastError());
  return 0;
}

// the upper sweep a call takes: 3 culled, 2 matrix cores, 0 VALU
// (O3DX_RANSAC_UPPER=cull / mfma2 / valu: test hook forcing one of them)
static int upper_mode(int64_t n, double smax, double thr) {
  if (const char* ue = getenv("O3DX_RANSAC_UPPER")) {
    if (std::strcmp(ue, "cull") == 0) return 3;
    if (std::strcmp(ue, "mfma2") == 0) return 2;
    return 0;
  }
  if (n >= kCullMinN) return 3;
  return std::ldexp(1.0, MfmaShape<true>::kBoundExp) * smax <= 0.02 * thr ? 2 : 0;
}

// Upper bounds of the counts (k_plane_upper); degenerate hypotheses -1.
static int run_count_upper(const float* xyz, int64_t n, const double* planes, int H, double thr, CountWs& w,
                           void* aabb_ws, double* mm_dev, hipStream_t s, std::vector<int64_t>& ub,
                           const double* absmax_in = nullptr, bool mm_ready = false) {
  double absmax[3];
  if (absmax_in) std::memcpy(absmax, absmax_in, sizeof(absmax));
  else {
    O3DX_TRY(absmax_of(xyz, n, aabb_ws, mm_dev, s, absmax));
    mm_ready = true;
  }
  std::vector<float4> p32;
  std::vector<float4> bnd;
  std::vector<uint8_t> dg;
  std::vector<uint8_t> st;
  int rc;
  double hmax;
  // The matrix-core sweep (two MFMAs, band thr + 2^-17 S_h) is wider than the
  // VALU sweep's (thr + 6 2^-24 S_h): it is used while its band adds at most
  // 2 % to thr, so the bounds stay about as tight and the replay consults
  // about as many hypotheses.
  double smax = 0.0;
  for (int h = 0; h < H; ++h) {
    const double* pl = planes + 4 * h;
    const double S = std::fabs(pl[0]) * absmax[0] + std::fabs(pl[1]) * absmax[1] + std::fabs(pl[2]) * absmax[2] +
                     std::fabs(pl[3]);
    if (std::isfinite(S)) smax = std::max(smax, S);
  }
  int mfma = upper_mode(n, smax, thr);
  // the culled sweep's sure band needs thr - g_h > 0; tiny thresholds (or
  // non-finite bounds) take the dense sweeps
  if (mfma == 3 && !(6.0 * std::ldexp(1.0, -24) * smax + std::ldexp(1.0, -20) * thr < 0.5 * thr))
    mfma = std::ldexp(1.0, MfmaShape<true>::kBoundExp) * smax <= 0.02 * thr ? 2 : 0;
  if (mfma == 3 && !w.binned) {
    if (!mm_ready) O3DX_TRY(aabb_device(xyz, n, mm_dev, aabb_ws, s));
    O3DX_TRY(bin_points(xyz, n, mm_dev, w, s));
  }
  upload_planes(planes, H, absmax, thr, w, p32, bnd, dg, st, s, &rc, &hmax, mfma);
  if (rc) return rc;
  KTimer kt("plane_count_upper", s);
  if (mfma == 3) {
    O3DX_TRY(launch_cull(n, H, w, s, w.counts));
    kt.stop();
    ub.resize(H);
    O3DX_TRY(read_back(ub.data(), w.counts, H * sizeof(int64_t), s));
    return 0;
  }
  if (mfma) {
    const int nch = (H + 31) / 32;
    auto launch_mfma = [&](auto kern, int tiles, int chunks) {
      const int ngy = (nch + chunks - 1) / chunks;
      const int64_t nbat = std::max<int64_t>(1, (n + 32 * tiles - 1) / (32 * tiles));
      // ~4 batches per wave, at most 2048 point blocks (the partial rows)
      const int64_t nbx = std::min<int64_t>(2048, std::max<int64_t>(1, (nbat + 15) / 16));
      const int64_t bpb = (nbat + nbx - 1) / nbx;
      const unsigned gx = (unsigned)((nbat + bpb - 1) / bpb);
      hipLaunchKernelGGL(kern, dim3(gx, ngy), dim3(kBlock), 0, s, xyz, n, w.mfrag, w.mhi, nch, H, bpb, w.partial);
      return gx;
    };
    const unsigned gx = launch_mfma(k_plane_upper_mfma<true>, MfmaShape<true>::kTiles, MfmaShape<true>::kChunks);
    O3DX_TRY(reduce_columns_i32_to_i64(w.partial, gx, H, w.counts, s));
    hipLaunchKernelGGL(k_mark_degenerate, dim3((H + 255) / 256), dim3(256), 0, s, w.degen, H, w.counts);
    kt.stop();
    ub.resize(H);
    O3DX_TRY(read_back(ub.data(), w.counts, H * sizeof(int64_t), s));
    O3DX_HIP(hipGetLastError());
    return 0;
  }
  // hi >= thr + g of every hypothesis (rounded up; nothing counted without any)
  float hi = (float)hmax;
  if ((double)hi < hmax) hi = std::nextafter(hi, INFINITY);
  if (hmax < 0) hi = -1.0f;
  constexpr int hc = 32, pl = 16;
  int nwp;
  int64_t bpw;
  const int nchunks = (H + hc - 1) / hc;
  count_geometry(n, 64 * pl, &nwp, &bpw, nchunks, H, w.partial_ints);
  const int ncg = (nchunks + kBlock / 64 - 1) / (kBlock / 64);
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)(nwp * ncg)), dim3(kBlock), 0, s, xyz, n, w.pl32, H, hi, bpw, nwp, ncg,
                       w.partial);
  };
  launch(k_plane_upper<hc, pl>);
  O3DX_TRY(reduce_columns_i32_to_i64(w.partial, nwp, H, w.counts, s));
  hipLaunchKernelGGL(k_mark_degenerate, dim3((H + 255) / 256), dim3(256), 0, s, w.degen, H, w.counts);
  kt.stop();
  ub.resize(H);
  O3DX_TRY(read_back(ub.data(), w.counts, H * sizeof(int64_t), s));
  O3DX_HIP(hipGetLastError());
  return 0;
}

// Sigma |d| of the hypotheses `which` (exact fx sums; fx_host: {lo, hi, q, 0}
// rows, nullable), their float64 values into sums_host.
template <class T>
static int run_abs_sum(const T* xyz, int64_t n, const double* planes, const int32_t* which, int L, double thr,
                       CountWs& w, hipStream_t s, double* sums_host, int64_t* fx_host = nullptr) {
  if (L == 0) return 0;
  std::vector<double> sel((size_t)4 * L);
  for (int j = 0; j < L; ++j)
    for (int a = 0; a < 4; ++a) sel[4 * j + a] = planes[4 * which[j] + a];
  O3DX_HIP(hipMemcpyAsync(w.pl64, sel.data(), sel.size() * sizeof(double), hipMemcpyHostToDevice, s));
  const int bx = abs_sum_blocks(n);
  const int q = fx_exp(thr);
  hipLaunchKernelGGL(k_plane_abs_sum<T>, dim3(bx, L), dim3(kBlock), 0, s, xyz, n, w.pl64, thr, fx_scale(q),
                     w.sum_partial);
  std::vector<int64_t> part((size_t)2 * bx * L);
  O3DX_TRY(read_back(part.data(), w.sum_partial, part.size() * sizeof(int64_t), s));
  O3DX_HIP(hipGetLastError());
  std::vector<int64_t> fx((size_t)4 * L);
  for (int j = 0; j < L; ++j) {
    int64_t lo = 0, hi = 0;  // integer sums: any order
    for (int b = 0; b < bx; ++b) {
      lo += part[2 * ((size_t)j * bx + b)];
      hi += part[2 * ((size_t)j * bx + b) + 1];
    }
    fx[4 * j] = lo;
    fx[4 * j + 1] = hi;
    fx[4 * j + 2] = q;
    fx[4 * j + 3] = 0;
  }
  fx_to_double(fx.data(), L, sums_host);
  if (fx_host) std::memcpy(fx_host, fx.data(), fx.size() * sizeof(int64_t));
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

// The hypotheses whose rmse select_best can consult.  Its running best count
// (and with it the early-break point) follows from the counts alone — rmse
// only decides WHICH of equal-count hypotheses is the best — so a replay on
// the counts finds every comparison "fit == best_fit && rmse < best_rmse": the
// hypotheses processed while their count equals the running maximum, for
// every maximum reached by at least two of them.  Usually the best count is
// unique and no Sigma |d| pass is needed at all.
static std::vector<int32_t> tied_hypotheses(const std::vector<int64_t>& counts, const double* planes, int64_t n,
                                            int ransac_n, double probability) {
  const int H = (int)counts.size();
  std::vector<int32_t> out, run;  // run: the hypotheses at the current running maximum
  int64_t best = 0;
  size_t break_iteration = std::numeric_limits<size_t>::max();
  int iteration_count = 0;
  auto flush = [&]() {
    if (run.size() >= 2) out.insert(out.end(), run.begin(), run.end());
    run.clear();
  };
  for (int it = 0; it < H; ++it) {
    if ((size_t)iteration_count > break_iteration) continue;
    if (counts[it] < 0 || (planes && plane_is_zero(planes + 4 * it))) continue;
    if (counts[it] > 0 && counts[it] >= best) {
      if (counts[it] > best) {
        flush();
        best = counts[it];
        const double fit = (double)best / (double)n;
        if (fit < 1.0) {
          double bi = std::min(std::log(1 - probability) / std::log(1 - std::pow(fit, ransac_n)), (double)H);
          break_iteration = (size_t)bi;
        } else {
          break_iteration = 0;
        }
      }
      run.push_back(it);
    }
    iteration_count++;
  }
  flush();
  std::sort(out.begin(), out.end());
  return out;
}

// Which hypotheses still need an exact count before the selection is
// decided.  v: exact counts where known[h], upper bounds elsewhere.  The
// replay of select_best / tied_hypotheses on v consults a hypothesis's count
// only when it is a record or a tie (v > 0 and v >= the running best); an
// unknown one outside those positions has exact <= ub < best (or ub == 0), so
// the exact replay skips it too, with the same running best and early break.
// Empty result: every consulted count is exact, and replays on v decide as
// on the exact counts.  Otherwise the unknown records/ties of this replay
// (speculative: the ones a later replay may still add are few).
static std::vector<int32_t> needed_exact(const int64_t* v, const uint8_t* known, const double* planes, int H,
                                         int64_t n, int ransac_n, double probability) {
  std::vector<int32_t> out;
  int64_t best = 0;
  size_t break_iteration = std::numeric_limits<size_t>::max();
  int iteration_count = 0;
  for (int it = 0; it < H; ++it) {
    if ((size_t)iteration_count > break_iteration) continue;
    if (v[it] < 0 || (planes && plane_is_zero(planes + 4 * it))) continue;
    if (v[it] > 0 && v[it] >= best) {
      if (!known[it]) out.push_back(it);
      if (v[it] > best) {
        best = v[it];
        const double fit = (double)best / (double)n;
        if (fit < 1.0) {
          double bi = std::min(std::log(1 - probability) / std::log(1 - std::pow(fit, ransac_n)), (double)H);
          break_iteration = (size_t)bi;
        } else {
          break_iteration = 0;
        }
      }
    }
    iteration_count++;
  }
  return out;
}

// moments pass (fx sums, common.hpp) over idx[0..m) (or the first m points);
// A bounds |coordinate|; out: 3 (pass 1) or 6 (pass 2) float64; fx_host
// (nullable): their {lo, hi, q, 0} rows
static int run_moments(const float* xyz, const int32_t* idx, int64_t m, const double* centroid, double A,
                       int64_t* part, int64_t* out_dev, hipStream_t s, double out[6], int64_t* fx_host = nullptr) {
  const int K = centroid ? 6 : 3;
  int q[6];
  mom_fx_exps(A, centroid != nullptr, q);
  int64_t digits[12] = {0}, fx[24];
  if (m > 0) {
    const int nb = mom_blocks(m);
    MomScales sc;
    for (int k = 0; k < 6; ++k) sc.s[k] = fx_scale(q[k]);
    hipLaunchKernelGGL(k_plane_moments<float>, dim3(nb), dim3(kBlock), 0, s, xyz, idx, m, centroid ? centroid[0] : 0.0,
                       centroid ? centroid[1] : 0.0, centroid ? centroid[2] : 0.0, centroid ? 1 : 0, sc, part);
    O3DX_TRY(reduce_columns_i64(part, nb, 12, out_dev, s));
    O3DX_TRY(read_back(digits, out_dev, sizeof(digits), s));
    O3DX_HIP(hipGetLastError());
  }
  fx_pack(digits, q, K, fx);
  fx_to_double(fx, K, out);
  if (fx_host) std::memcpy(fx_host, fx, (size_t)4 * K * sizeof(int64_t));
  return 0;
}

// ------------------------------------------------------ float64 clouds
// Exact counts on float64 coordinates (the float64 boundary,
// o3dx_segment_plane_f64): every (point, hypothesis) pair evaluated as
// Open3D evaluates it on its float64 storage, |(a x + c z) + (b y + d)| < thr
// (plane_dist64).  A lane holds kC64Pts points; the block's kC64HC planes sit
// in LDS (broadcast reads); per hypothesis a wave adds the ballot counts of
// its points into an LDS counter; partial[bx][H] per block, int32.
constexpr int kC64Pts = 4;
constexpr int kC64HC = 64;
constexpr int kC64MaxBlocks = 2048;  // <= CountWs::partial_ints / H rows

__global__ void __launch_bounds__(kBlock) k_plane_count64(const double* __restrict__ xyz, int64_t n,
                                                          const double* __restrict__ pl64, int H, double thr,
                                                          int32_t* __restrict__ partial) {
  __shared__ double pl[kC64HC][4];
  __shared__ int cnt[kC64HC];
  const int h0 = blockIdx.y * kC64HC, hc = min(kC64HC, H - h0);
  for (int t = threadIdx.x; t < kC64HC * 4; t += kBlock) pl[t >> 2][t & 3] = t < hc * 4 ? pl64[4 * (int64_t)h0 + t] : 0.0;
  for (int t = threadIdx.x; t < kC64HC; t += kBlock) cnt[t] = 0;
  __syncthreads();
  const int64_t tile = (int64_t)kBlock * kC64Pts;
  for (int64_t base = (int64_t)blockIdx.x * tile; base < n; base += (int64_t)gridDim.x * tile) {
    double X[kC64Pts], Y[kC64Pts], Z[kC64Pts];
#pragma unroll
    for (int k = 0; k < kC64Pts; ++k) {
      const int64_t i = base + threadIdx.x + (int64_t)k * kBlock;
      if (i < n) {
        load3(xyz, i, X[k], Y[k], Z[k]);
      } else {
        X[k] = Y[k] = Z[k] = __longlong_as_double(0x7ff8000000000000ll);  // NaN: never counted
      }
    }
    for (int h = 0; h < hc; ++h) {
      int c = 0;
#pragma unroll
      for (int k = 0; k < kC64Pts; ++k) c += __popcll(__ballot(plane_dist64(pl[h], X[k], Y[k], Z[k]) < thr));
      if ((threadIdx.x & 63) == 0 && c) atomicAdd(&cnt[h], c);
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < hc; t += kBlock) partial[(int64_t)blockIdx.x * H + h0 + t] = cnt[t];
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
  int64_t* mom_part;
  int64_t* mom_part2;
  int64_t* mom_out;
  int64_t* fin;  // {inlier count, pad, first sums (6), second sums (12)}
  char* rb;       // the culled path's read-back block: counts (8 H), float64 planes (32 H), bounds (48)
};

static size_t seg_carve(Arena& ar, int64_t n, int H, int rn, SegWs* w) {
  count_carve(ar, n, H, &w->cw);
  w->sidx = ar.take<int32_t>((size_t)H * rn);
  // sampled coordinates and the cloud's min/max side by side: one read-back
  const size_t nsc = ((size_t)H * rn * 3 + 1) & ~size_t(1);
  w->scoord = ar.take<float>(nsc + 16);
  w->mm = reinterpret_cast<double*>(w->scoord + nsc);
  w->flags = ar.take<uint8_t>(n + 16);
  w->scan_tmp = ar.take<int32_t>(compact_workspace_ints(n));
  w->aabb = ar.take<char>(aabb_ws_bytes(n));
  w->cnt = ar.take<int64_t>(4);
  w->mom_part = ar.take<int64_t>((size_t)std::max<int64_t>(mom_blocks(n) * 12, (int64_t)grid_for(n, kBlock, 8192) * 6));
  w->mom_part2 = ar.take<int64_t>((size_t)mom_blocks(n) * 12);
  w->mom_out = ar.take<int64_t>(16);
  w->fin = ar.take<int64_t>(24);
  w->rb = ar.take<char>(40 * (size_t)H + 64);
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

extern "C" int o3dx_planes_from_samples(const double* coords, int H, int ransac_n, double* planes) {
  if (H < 0 || ransac_n < 3 || (H > 0 && (!coords || !planes)))
    return fail(O3DX_EINVAL, "o3dx_planes_from_samples: bad arguments");
  for (int h = 0; h < H; ++h) plane_from_pts(coords + (size_t)h * ransac_n * 3, ransac_n, planes + 4 * (size_t)h);
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

extern "C" int o3dx_plane_count_upper(const float* xyz, int64_t n, const double* planes, int H, double thr,
                                      const double* absmax, int64_t* counts, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || H < 0 || (H > 0 && (!planes || !counts)) || (n > 0 && !xyz))
    return fail(O3DX_EINVAL, "o3dx_plane_count_upper: bad arguments");
  if (!ws || ws_bytes < o3dx_plane_count_workspace_bytes(n, H)) return fail(O3DX_ENOMEM, "count workspace too small");
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
  O3DX_TRY(run_count_upper(xyz, n, planes, H, thr, w, aabb, mm, s, c, absmax));
  std::memcpy(counts, c.data(), H * sizeof(int64_t));
  return 0;
}

extern "C" int o3dx_ransac_needed(const int64_t* counts, const uint8_t* known, const double* planes, int H, int64_t n,
                                  int ransac_n, double probability, int32_t* out, int32_t* n_out) {
  if (!counts || !known || !out || !n_out || H < 0 || n <= 0) return fail(O3DX_EINVAL, "o3dx_ransac_needed: bad args");
  const std::vector<int32_t> t = needed_exact(counts, known, planes, H, n, ransac_n, probability);
  std::memcpy(out, t.data(), t.size() * sizeof(int32_t));
  *n_out = (int32_t)t.size();
  return 0;
}

extern "C" int o3dx_plane_abs_sum(const float* xyz, int64_t n, const double* planes, const int32_t* which, int L,
                                  double thr, double* sums, int64_t* fx_out, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || L < 0 || (L > 0 && (!planes || !which || !sums))) return fail(O3DX_EINVAL, "o3dx_plane_abs_sum: bad args");
  if (!ws || ws_bytes < o3dx_plane_count_workspace_bytes(n, L)) return fail(O3DX_ENOMEM, "abs_sum workspace too small");
  if (L == 0) return 0;
  if (n == 0) {
    for (int j = 0; j < L; ++j) {
      sums[j] = 0;
      if (fx_out) {
        fx_out[4 * j] = fx_out[4 * j + 1] = fx_out[4 * j + 3] = 0;
        fx_out[4 * j + 2] = fx_exp(thr);
      }
    }
    return 0;
  }
  Arena ar(ws, ws_bytes);
  CountWs w;
  count_carve(ar, n, L, &w);
  O3DX_ARENA_CHECK(ar);
  return run_abs_sum(xyz, n, planes, which, L, thr, w, as_stream(stream), sums, fx_out);
}

extern "C" int o3dx_ransac_tied(const int64_t* counts, const double* planes, int H, int64_t n, int ransac_n,
                                double probability, int32_t* out, int32_t* n_out) {
  if (!counts || !out || !n_out || H < 0 || n <= 0) return fail(O3DX_EINVAL, "o3dx_ransac_tied: bad args");
  std::vector<int64_t> c(counts, counts + H);
  const std::vector<int32_t> t = tied_hypotheses(c, planes, n, ransac_n, probability);
  std::memcpy(out, t.data(), t.size() * sizeof(int32_t));
  *n_out = (int32_t)t.size();
  return 0;
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
  hipLaunchKernelGGL(k_plane_flags<float>, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, plane[0], plane[1],
                     plane[2], plane[3], thr, flags);
  O3DX_TRY(compact_flags(flags, n, idx_out, nullptr, cnt, tmp, s));
  O3DX_TRY(read_back(count_host, cnt, sizeof(int64_t), s));
  return 0;
}

extern "C" size_t o3dx_plane_select_workspace_bytes(int64_t n) {
  return Arena::align(n + 17) + Arena::align(compact_workspace_ints(n) * 4 + 1) + 512;
}

template <class T>
static int plane_select_impl(const T* xyz, int64_t n, const double* plane, int band, double lo, double hi, int invert,
                             double* dist_out, int32_t* idx_out, int64_t* count_host, void* ws, size_t ws_bytes,
                             void* stream) {
  if (n < 0 || !plane || (n > 0 && !xyz) || (idx_out && !count_host) || (!idx_out && !dist_out))
    return fail(O3DX_EINVAL, "o3dx_plane_select: bad args");
  if (idx_out && (!ws || ws_bytes < o3dx_plane_select_workspace_bytes(n)))
    return fail(O3DX_ENOMEM, "plane_select workspace too small");
  if (n == 0) {
    if (count_host) *count_host = 0;
    return 0;
  }
  // (a**2 + b**2 + c**2) ** 0.5 (Python: correctly rounded squares, left-to-right sum)
  const double nrm = std::sqrt(plane[0] * plane[0] + plane[1] * plane[1] + plane[2] * plane[2]);
  hipStream_t s = as_stream(stream);
  uint8_t* flags = nullptr;
  int32_t* tmp = nullptr;
  int64_t* cnt = nullptr;
  if (idx_out) {
    Arena ar(ws, ws_bytes);
    flags = ar.take<uint8_t>(n + 16);
    tmp = ar.take<int32_t>(compact_workspace_ints(n));
    cnt = ar.take<int64_t>(2);
    O3DX_ARENA_CHECK(ar);
  }
  const unsigned g = grid_for(n, kBlock, 8192);
  if (band)
    hipLaunchKernelGGL((k_plane_band<true, T>), dim3(g), dim3(kBlock), 0, s, xyz, n, plane[0], plane[1], plane[2],
                       plane[3], nrm, lo, hi, invert, flags, dist_out);
  else
    hipLaunchKernelGGL((k_plane_band<false, T>), dim3(g), dim3(kBlock), 0, s, xyz, n, plane[0], plane[1], plane[2],
                       plane[3], nrm, lo, hi, invert, flags, dist_out);
  O3DX_HIP(hipGetLastError());
  if (idx_out) {
    O3DX_TRY(compact_flags(flags, n, idx_out, nullptr, cnt, tmp, s));
    O3DX_TRY(read_back(count_host, cnt, sizeof(int64_t), s));
  }
  return 0;
}

extern "C" int o3dx_plane_select(const float* xyz, int64_t n, const double* plane, int band, double lo, double hi,
                                 int invert, double* dist_out, int32_t* idx_out, int64_t* count_host, void* ws,
                                 size_t ws_bytes, void* stream) {
  return plane_select_impl(xyz, n, plane, band, lo, hi, invert, dist_out, idx_out, count_host, ws, ws_bytes, stream);
}

extern "C" int o3dx_plane_select_f64(const double* xyz, int64_t n, const double* plane, int band, double lo,
                                     double hi, int invert, double* dist_out, int32_t* idx_out, int64_t* count_host,
                                     void* ws, size_t ws_bytes, void* stream) {
  return plane_select_impl(xyz, n, plane, band, lo, hi, invert, dist_out, idx_out, count_host, ws, ws_bytes, stream);
}

__global__ void __launch_bounds__(kBlock) k_absmax_sel(const float* __restrict__ xyz, const int32_t* __restrict__ idx,
                                                       int64_t m, unsigned int* __restrict__ out) {
  float a[3] = {0.f, 0.f, 0.f};
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx ? idx[j] : j;
    for (int c = 0; c < 3; ++c) a[c] = fmaxf(a[c], fabsf(xyz[3 * i + c]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int c = 0; c < 3; ++c) a[c] = fmaxf(a[c], __shfl_xor(a[c], o, 64));
  if ((threadIdx.x & 63) == 0)
    for (int c = 0; c < 3; ++c) atomicMax(&out[c], __float_as_uint(a[c]));  // non-negative: bits order as values
}

extern "C" size_t o3dx_plane_moments_workspace_bytes(int64_t count) {
  return Arena::align((size_t)mom_blocks(std::max<int64_t>(count, 1)) * 12 * sizeof(int64_t) + 1) + 1024;
}

extern "C" int o3dx_plane_moments(const float* xyz, const int32_t* idx, int64_t count, const double* centroid,
                                  const double* absmax, double* sums, int64_t* fx_out, void* ws, size_t ws_bytes,
                                  void* stream) {
  if (count < 0 || !sums || (count > 0 && !xyz)) return fail(O3DX_EINVAL, "o3dx_plane_moments: bad args");
  if (!ws || ws_bytes < o3dx_plane_moments_workspace_bytes(count))
    return fail(O3DX_ENOMEM, "moments workspace too small");
  hipStream_t s = as_stream(stream);
  Arena ar(ws, ws_bytes);
  int64_t* part = ar.take<int64_t>((size_t)mom_blocks(std::max<int64_t>(count, 1)) * 12);
  int64_t* outd = ar.take<int64_t>(16);
  double A = 0.0;
  if (absmax) {
    A = std::max(absmax[0], std::max(absmax[1], absmax[2]));
  } else if (count > 0) {  // the selected points' own bound
    unsigned int* u = reinterpret_cast<unsigned int*>(outd);
    O3DX_HIP(hipMemsetAsync(u, 0, 4 * sizeof(unsigned int), s));
    hipLaunchKernelGGL(k_absmax_sel, dim3(grid_for(count, kBlock, 1024)), dim3(kBlock), 0, s, xyz, idx, count, u);
    unsigned int b[4];
    O3DX_TRY(read_back(b, u, sizeof(b), s));
    for (int c = 0; c < 3; ++c) {
      float f;
      std::memcpy(&f, &b[c], 4);
      A = std::max(A, (double)f);
    }
  }
  double tmp[6];
  O3DX_TRY(run_moments(xyz, idx, count, centroid, A, part, outd, s, tmp, fx_out));
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
    hipLaunchKernelGGL(k_gather_samples<float>, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, xyz, w.sidx, ns, w.scoord);
  }
  // |x|,|y|,|z| bounds of the cloud: the count's float32 window and the fx
  // quantum of the refit moments (a sharded driver passes the global ones)
  O3DX_TRY(aabb_device(xyz, n, w.mm, w.aabb, s));
  double absmax[3];
  std::vector<int64_t> counts;
  const bool device_setup = H > 0 && upper_mode(n, 0.0, thr) == 3 && !getenv("O3DX_RANSAC_HOST_SETUP");
  if (device_setup) {
    // the culled path without a host round trip before the sweep: Morton
    // order, the hypotheses and their limits on the device (k_ransac_setup,
    // the host's own plane math), the sweep; then {counts, float64 planes,
    // bounds} come back in one read
    O3DX_TRY(bin_points(xyz, n, w.mm, w.cw, s));
    int64_t* rb_counts = reinterpret_cast<int64_t*>(w.rb);
    double* rb_pl64 = reinterpret_cast<double*>(w.rb + 8 * (size_t)H);
    double* rb_mm = reinterpret_cast<double*>(w.rb + 40 * (size_t)H);
    hipLaunchKernelGGL(k_ransac_setup, dim3((unsigned)((H + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, w.scoord, H,
                       ransac_n, w.mm, thr, w.cw.pl32, w.cw.band, w.cw.degen, rb_pl64, rb_mm);
    // the sweep's own tables (pl64 is read only by the exact form): the upload block's
    {
      KTimer kt("plane_count_upper", s);
      O3DX_TRY(launch_cull(n, H, w.cw, s, rb_counts));
    }
    std::vector<char> rb(40 * (size_t)H + 6 * sizeof(double));
    O3DX_TRY(read_back(rb.data(), w.rb, rb.size(), s));
    counts.resize(H);
    std::memcpy(counts.data(), rb.data(), 8 * (size_t)H);
    std::memcpy(planes.data(), rb.data() + 8 * (size_t)H, 32 * (size_t)H);
    double mmh[6];
    std::memcpy(mmh, rb.data() + 40 * (size_t)H, sizeof(mmh));
    for (int a = 0; a < 3; ++a) absmax[a] = std::max(std::fabs(mmh[a]), std::fabs(mmh[3 + a]));
    // run_count_upper's guard on the culled sweep, replayed on the returned
    // bounds: a threshold tiny against the coordinates leaves the culled
    // bounds loose (valid, but the replay would then count many hypotheses
    // exactly); such inputs take the dense sweep instead
    double smax = 0.0;
    for (int h = 0; h < H; ++h) {
      const double* pl = &planes[(size_t)4 * h];
      const double S = std::fabs(pl[0]) * absmax[0] + std::fabs(pl[1]) * absmax[1] + std::fabs(pl[2]) * absmax[2] +
                       std::fabs(pl[3]);
      if (std::isfinite(S)) smax = std::max(smax, S);
    }
    if (!(6.0 * std::ldexp(1.0, -24) * smax + std::ldexp(1.0, -20) * thr < 0.5 * thr))
      O3DX_TRY(run_count_upper(xyz, n, planes.data(), H, thr, w.cw, w.aabb, w.mm, s, counts, absmax, true));
  } else {
    // read back together with the sampled coordinates
    const size_t off_mm = reinterpret_cast<char*>(w.mm) - reinterpret_cast<char*>(w.scoord);
    std::vector<char> rb(off_mm + 6 * sizeof(double));
    O3DX_TRY(read_back(rb.data(), w.scoord, rb.size(), s));
    {
      double mmh[6];
      std::memcpy(mmh, rb.data() + off_mm, sizeof(mmh));
      for (int a = 0; a < 3; ++a) absmax[a] = std::max(std::fabs(mmh[a]), std::fabs(mmh[3 + a]));
    }
    // the culled sweep's Morton order: queued now, it runs while the host
    // computes the hypotheses
    if (H > 0 && upper_mode(n, 0.0, thr) == 3) O3DX_TRY(bin_points(xyz, n, w.mm, w.cw, s));
    if (H > 0) {
      const float* sc = reinterpret_cast<const float*>(rb.data());
      std::vector<double> P((size_t)ransac_n * 3);
      for (int h = 0; h < H; ++h) {
        for (int j = 0; j < ransac_n * 3; ++j) P[j] = (double)sc[(size_t)h * ransac_n * 3 + j];
        plane_from_pts(P.data(), ransac_n, &planes[(size_t)4 * h]);
      }
    }
  }
  const double A = std::max(absmax[0], std::max(absmax[1], absmax[2]));
  int best = -1;
  if (H > 0) {
    // upper bounds for all, exact counts for the hypotheses the replay consults
    if (!device_setup)
      O3DX_TRY(run_count_upper(xyz, n, planes.data(), H, thr, w.cw, w.aabb, w.mm, s, counts, absmax, true));
    std::vector<uint8_t> known(H, 0);
    std::vector<double> sub;
    std::vector<int64_t> ec;
    for (;;) {
      const std::vector<int32_t> need =
          needed_exact(counts.data(), known.data(), planes.data(), H, n, ransac_n, probability);
      if (need.empty()) break;
      const int L = (int)need.size();
      sub.resize((size_t)4 * L);
      for (int j = 0; j < L; ++j) std::memcpy(&sub[(size_t)4 * j], &planes[(size_t)4 * need[j]], 4 * sizeof(double));
      O3DX_TRY(run_count(xyz, n, sub.data(), L, thr, w.cw, w.aabb, w.mm, s, ec, absmax));
      for (int j = 0; j < L; ++j) {
        counts[need[j]] = ec[j];
        known[need[j]] = 1;
      }
    }
    std::vector<int32_t> tied = tied_hypotheses(counts, planes.data(), n, ransac_n, probability);
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
  // the inliers and GetPlaneFromPoints over them with one host wait: flags +
  // first moments (one read of the cloud), compaction, the centroid and the
  // second moments on the device; then {k, first sums, second sums} back
  int64_t fin[20] = {0};
  int q1[6], q2[6];
  mom_fx_exps(A, false, q1);
  mom_fx_exps(A, true, q2);
  if (!plane_is_zero(bp)) {
    MomScales sc1, sc2;
    for (int a = 0; a < 6; ++a) {
      sc1.s[a] = fx_scale(q1[a]);
      sc2.s[a] = fx_scale(q2[a]);
    }
    const unsigned gf = grid_for(n, kBlock, 8192);
    hipLaunchKernelGGL(k_plane_flags_sum<float>, dim3(gf), dim3(kBlock), 0, s, xyz, n, bp[0], bp[1], bp[2], bp[3], thr, sc1,
                       w.flags, w.mom_part);
    O3DX_TRY(compact_flags(w.flags, n, inliers_out, nullptr, w.fin, w.scan_tmp, s));
    O3DX_TRY(reduce_columns_i64(w.mom_part, gf, 6, w.fin + 2, s));
    const int nb2 = mom_blocks(n);
    hipLaunchKernelGGL(k_plane_moments_c<float>, dim3(nb2), dim3(kBlock), 0, s, xyz, inliers_out, w.fin, w.fin + 2, q1[0],
                       q1[1], q1[2], sc2, w.mom_part2);
    O3DX_TRY(reduce_columns_i64(w.mom_part2, nb2, 12, w.fin + 8, s));
    O3DX_HIP(hipGetLastError());
    O3DX_TRY(read_back(fin, w.fin, sizeof(fin), s));
  }
  const int64_t k = fin[0];
  *n_inliers_host = k;
  // GetPlaneFromPoints over the final inliers (zero plane when there are none)
  if (k == 0) {
    for (int a = 0; a < 4; ++a) plane_host[a] = 0;
    return 0;
  }
  int64_t fx[24];
  double s1[6], s2[6], c[3];
  fx_pack(fin + 2, q1, 3, fx);
  fx_to_double(fx, 3, s1);
  for (int a = 0; a < 3; ++a) c[a] = s1[a] / (double)k;
  fx_pack(fin + 8, q2, 6, fx);
  fx_to_double(fx, 6, s2);
  plane_from_centred(c, s2, plane_host);
  return 0;
}

// ------------------------------------------------------ float64 boundary
// segment_plane on float64 coordinates (LAS / E57-style clouds the float32
// path would round, reference PointCloud.py:75-77 on the float64 storage of
// :99-102): the hypotheses from the float64 samples (the host's plane math),
// exact counts of every hypothesis (k_plane_count64; no upper-bound sweep),
// Open3D's replay (select_best, Sigma|d| for the ties), then the inliers and
// the GetPlaneFromPoints refit over them as on the float32 path.
extern "C" size_t o3dx_segment_plane_f64_workspace_bytes(int64_t n, int iters) {
  return o3dx_segment_plane_workspace_bytes(n, iters) + Arena::align((size_t)std::max(iters, 1) * 16 * 3 * 8 + 64) +
         Arena::align(aabb64_ws_bytes() + 64) + 1024;
}

static int count64(const double* xyz, int64_t n, const double* planes, int H, double thr, CountWs& w, hipStream_t s,
                   std::vector<int64_t>& counts) {
  counts.assign(H, 0);
  if (H == 0) return 0;
  O3DX_HIP(hipMemcpyAsync(w.pl64, planes, (size_t)4 * H * sizeof(double), hipMemcpyHostToDevice, s));
  const int64_t tiles = (n + (int64_t)kBlock * kC64Pts - 1) / ((int64_t)kBlock * kC64Pts);
  const int rows = (int)std::max<int64_t>(1, std::min<int64_t>({tiles, (int64_t)kC64MaxBlocks,
                                                                 (int64_t)(w.partial_ints / (size_t)H)}));
  KTimer kt("plane_count", s);
  if (n > 0) {
    hipLaunchKernelGGL(k_plane_count64, dim3((unsigned)rows, (unsigned)((H + kC64HC - 1) / kC64HC)), dim3(kBlock), 0,
                       s, xyz, n, w.pl64, H, thr, w.partial);
    O3DX_TRY(reduce_columns_i32_to_i64(w.partial, rows, H, w.counts, s));
    O3DX_TRY(read_back(counts.data(), w.counts, (size_t)H * sizeof(int64_t), s));
  }
  O3DX_HIP(hipGetLastError());
  for (int h = 0; h < H; ++h)
    if (plane_is_zero(planes + 4 * (size_t)h)) counts[h] = -1;
  return 0;
}

extern "C" int o3dx_plane_count_f64(const double* xyz, int64_t n, const double* planes, int H, double thr,
                                    int64_t* counts, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || H < 0 || (n > 0 && !xyz) || (H > 0 && (!planes || !counts)))
    return fail(O3DX_EINVAL, "o3dx_plane_count_f64: bad arguments");
  if (!ws || ws_bytes < o3dx_plane_count_workspace_bytes(n, H)) return fail(O3DX_ENOMEM, "plane_count workspace too small");
  if (H == 0) return 0;
  Arena ar(ws, ws_bytes);
  CountWs w;
  count_carve(ar, n, H, &w);
  O3DX_ARENA_CHECK(ar);
  std::vector<int64_t> c;
  O3DX_TRY(count64(xyz, n, planes, H, thr, w, as_stream(stream), c));
  std::memcpy(counts, c.data(), (size_t)H * sizeof(int64_t));
  return 0;
}

extern "C" int o3dx_segment_plane_f64(const double* xyz, int64_t n, double thr, int ransac_n, int iters,
                                      double probability, const int32_t* samples_host, double* plane_host,
                                      int32_t* inliers_out, int64_t* n_inliers_host, void* ws, size_t ws_bytes,
                                      void* stream) {
  if (!(probability > 0.0 && probability <= 1.0)) return fail(O3DX_EINVAL, "Probability must be > 0 or <= 1.0");
  if (ransac_n < 3) return fail(O3DX_EINVAL, "ransac_n should be set to higher than or equal to 3.");
  if (n < ransac_n) return fail(O3DX_EINVAL, "There must be at least 'ransac_n' points.");
  if (ransac_n > 16) return fail(O3DX_ENOTSUP, "ransac_n > 16 not supported");
  if (iters < 0 || !plane_host || !n_inliers_host || !inliers_out || !xyz || (iters > 0 && !samples_host))
    return fail(O3DX_EINVAL, "o3dx_segment_plane_f64: bad arguments");
  if (!ws || ws_bytes < o3dx_segment_plane_f64_workspace_bytes(n, iters))
    return fail(O3DX_ENOMEM, "segment_plane workspace too small");
  hipStream_t s = as_stream(stream);
  const int H = iters;
  Arena ar(ws, ws_bytes);
  SegWs w;
  seg_carve(ar, n, std::max(H, 1), 16, &w);
  const size_t ncoord = (size_t)std::max(H, 1) * ransac_n * 3;
  double* sc64 = ar.take<double>(ncoord + 8);  // sampled coordinates, then the cloud's {min, max}
  double* mmd = sc64 + ncoord;
  char* aws = ar.take<char>(aabb64_ws_bytes() + 64);
  O3DX_ARENA_CHECK(ar);
  if (H > 0) {
    const int64_t ns = (int64_t)H * ransac_n;
    for (int64_t j = 0; j < ns; ++j)
      if (samples_host[j] < 0 || samples_host[j] >= n) return fail(O3DX_EINVAL, "sample index out of range");
    O3DX_HIP(hipMemcpyAsync(w.sidx, samples_host, ns * sizeof(int32_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_gather_samples<double>, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, xyz, w.sidx, ns,
                       sc64);
  }
  O3DX_TRY(aabb64_device(xyz, n, mmd, aws, s));
  std::vector<double> rb(ncoord + 6);
  O3DX_TRY(read_back(rb.data(), sc64, rb.size() * sizeof(double), s));
  double absmax[3];
  for (int a = 0; a < 3; ++a) absmax[a] = std::max(std::fabs(rb[ncoord + a]), std::fabs(rb[ncoord + 3 + a]));
  const double A = std::max(absmax[0], std::max(absmax[1], absmax[2]));
  std::vector<double> planes((size_t)4 * std::max(H, 1), 0.0);
  for (int h = 0; h < H; ++h) plane_from_pts(&rb[(size_t)h * ransac_n * 3], ransac_n, &planes[(size_t)4 * h]);
  int best = -1;
  if (H > 0) {
    std::vector<int64_t> counts;
    O3DX_TRY(count64(xyz, n, planes.data(), H, thr, w.cw, s, counts));
    std::vector<int32_t> tied = tied_hypotheses(counts, planes.data(), n, ransac_n, probability);
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
  int64_t fin[20] = {0};
  int q1[6], q2[6];
  mom_fx_exps(A, false, q1);
  double E = 0.0;
  for (int a = 0; a < 3; ++a) E = std::max(E, rb[ncoord + 3 + a] - rb[ncoord + a]);
  mom_fx_exps_span(E, q2);
  if (!plane_is_zero(bp)) {
    MomScales sc1, sc2;
    for (int a = 0; a < 6; ++a) {
      sc1.s[a] = fx_scale(q1[a]);
      sc2.s[a] = fx_scale(q2[a]);
    }
    const unsigned gf = grid_for(n, kBlock, 8192);
    hipLaunchKernelGGL(k_plane_flags_sum<double>, dim3(gf), dim3(kBlock), 0, s, xyz, n, bp[0], bp[1], bp[2], bp[3],
                       thr, sc1, w.flags, w.mom_part);
    O3DX_TRY(compact_flags(w.flags, n, inliers_out, nullptr, w.fin, w.scan_tmp, s));
    O3DX_TRY(reduce_columns_i64(w.mom_part, gf, 6, w.fin + 2, s));
    const int nb2 = mom_blocks(n);
    hipLaunchKernelGGL(k_plane_moments_c<double>, dim3(nb2), dim3(kBlock), 0, s, xyz, inliers_out, w.fin, w.fin + 2,
                       q1[0], q1[1], q1[2], sc2, w.mom_part2);
    O3DX_TRY(reduce_columns_i64(w.mom_part2, nb2, 12, w.fin + 8, s));
    O3DX_HIP(hipGetLastError());
    O3DX_TRY(read_back(fin, w.fin, sizeof(fin), s));
  }
  const int64_t k = fin[0];
  *n_inliers_host = k;
  if (k == 0) {
    for (int a = 0; a < 4; ++a) plane_host[a] = 0;
    return 0;
  }
  int64_t fx[24];
  double s1[6], s2[6], c[3];
  fx_pack(fin + 2, q1, 3, fx);
  fx_to_double(fx, 3, s1);
  for (int a = 0; a < 3; ++a) c[a] = s1[a] / (double)k;
  fx_pack(fin + 8, q2, 6, fx);
  fx_to_double(fx, 6, s2);
  plane_from_centred(c, s2, plane_host);
  return 0;
}
