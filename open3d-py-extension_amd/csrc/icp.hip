// icp.hip — point-to-plane ICP (north-star op; no symbol in the reference,
// attached as PointCloud.registration_icp / Processors.ICP).
//
// Semantics restated from Open3D pipelines/registration/Registration.cpp
// (RegistrationICP, GetRegistrationResultAndCorrespondences with
// SearchHybrid(p, max_corr, 1)), TransformationEstimation.cpp
// (PointToPlane::ComputeTransformation), utility/Eigen.cpp (ComputeJTJandJTr,
// SolveJacobianSystemAndObtainExtrinsicMatrix, TransformVector6dToMatrix4d).
//
// One fused pass per iteration: transform the float32 source by the float64
// cumulative T, nearest target within max_corr (target grid), residual
// r = (vs - vt).nt, J = [vs x nt ; nt], and a fixed-order float64 reduction
// of the 29 moments (21 JTJ + 6 JTr + r^2 + count, plus sum d^2) — per-lane,
// wave xor-tree, block, then block partials in block order.  The 6x6 solve
// and the loop stay on the host (float64 LDLT with diagonal pivoting).
#include <vector>

#include "grid.hpp"

namespace o3dx {

constexpr int kIcpBlocks = 1024;
constexpr int kNS = O3DX_ICP_NSUMS;

struct Mat4 {
  double m[16];
};

// One correspondence -> its 30 float64 moment terms: r = (vs - vt).nt,
// J = [vs x nt ; nt] (Open3D ComputeJTJandJTr order), plus count and d^2.
constexpr int kNT = 30;

__device__ __forceinline__ void icp_terms(double t[kNT], double px, double py, double pz, const float4 vt,
                                          const float4 nt, double d2) {
  const double nx = nt.x, ny = nt.y, nz = nt.z;
  const double r = ((px - (double)vt.x) * nx + (py - (double)vt.y) * ny) + (pz - (double)vt.z) * nz;
  double J[6];
  J[0] = py * nz - pz * ny;
  J[1] = pz * nx - px * nz;
  J[2] = px * ny - py * nx;
  J[3] = nx;
  J[4] = ny;
  J[5] = nz;
  int k = 0;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = a; b < 6; ++b) t[k++] = J[a] * J[b];
#pragma unroll
  for (int a = 0; a < 6; ++a) t[21 + a] = J[a] * r;
  t[27] = r * r;
  t[28] = 1.0;
  t[29] = d2;
}

// fx scales (2^-q) of the 30 sums, from bounds every rank derives alike
struct FxScales {
  double s[kNT];
};

// Source point j -> (original index, float64 position under T).  SORTED: src
// is float4 (x, y, z, bits(original index)) in the compact spatial order of
// o3dx_spatial_sort, so the 64 queries of a wave probe neighbouring target
// cells; else plain (n,3) float32 in caller order.
template <bool SORTED>
__device__ __forceinline__ int64_t icp_source(const float* __restrict__ src, int64_t j, const Mat4& T, double* px,
                                              double* py, double* pz) {
  double x, y, z;
  int64_t i;
  if (SORTED) {
    const float4 v = reinterpret_cast<const float4*>(src)[j];
    x = v.x;
    y = v.y;
    z = v.z;
    i = __float_as_int(v.w);
  } else {
    i = j;
    x = src[3 * i];
    y = src[3 * i + 1];
    z = src[3 * i + 2];
  }
  const double* t = T.m;
  // Eigen 4x4 * (x,y,z,1): ((T0 x + T1 y) + T2 z) + T3 per row
  *px = ((t[0] * x + t[1] * y) + t[2] * z) + t[3];
  *py = ((t[4] * x + t[5] * y) + t[6] * z) + t[7];
  *pz = ((t[8] * x + t[9] * y) + t[10] * z) + t[11];
  return i;
}

// Pass 1 — correspondences: one thread per source point, the 1-NN within
// max_correspondence_distance (nn_search_dev); writes the target's sorted
// position (-1: none) and, when asked, the target's original index by source
// index.  No accumulators live here, so the search runs at full occupancy
// (the search is latency-bound: many waves hide the dependent cell loads).
// ROWS: the search beyond the own cell walks (y, z) rows (nn_search_dev).
template <bool SORTED, bool ROWS>
__global__ void __launch_bounds__(kBlock) k_icp_match(const float* __restrict__ src, int64_t ns, GridView g, Mat4 T,
                                                      double radius, int32_t* __restrict__ mpos,
                                                      int32_t* __restrict__ cj) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ns) return;
  double px, py, pz;
  const int64_t i = icp_source<SORTED>(src, j, T, &px, &py, &pz);
  double d2;
  int pos;
  const int tj = nn_search_dev<ROWS>(g, px, py, pz, radius, &d2, &pos);
  mpos[j] = pos;
  if (cj) cj[i] = tj;
}

// Pass 2 — moments: a streaming pass over the matched pairs (source point,
// target point + normal gathered by sorted position), the 30 moment terms per
// pair as exact fx integers (common.hpp), summed per lane in int64, then per
// block into {lo, hi} digit partials: the sums are the same bits for any
// split of the source over lanes, blocks or ranks.  d^2 is recomputed exactly
// as the search computed it.
template <bool SORTED>
__global__ void __launch_bounds__(kBlock) k_icp_moments(const float* __restrict__ src, int64_t ns, GridView g,
                                                        const float4* __restrict__ tnorm, Mat4 T,
                                                        const int32_t* __restrict__ mpos, FxScales sc,
                                                        int64_t* __restrict__ partial) {
  __shared__ int64_t sh[(kBlock / 64) * 2 * kNT];
  int64_t acc[kNT];
#pragma unroll
  for (int k = 0; k < kNT; ++k) acc[k] = 0;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ns; j += (int64_t)gridDim.x * blockDim.x) {
    const int pos = mpos[j];
    if (pos < 0) continue;
    double px, py, pz;
    icp_source<SORTED>(src, j, T, &px, &py, &pz);
    const float4 vt = g.pts[pos];
    double t[kNT];
    icp_terms(t, px, py, pz, vt, tnorm[pos], dist2_f64(px, py, pz, vt));
#pragma unroll
    for (int k = 0; k < kNT; ++k) acc[k] += fx_term(t[k], sc.s[k]);
  }
  int64_t* out = partial + (int64_t)blockIdx.x * 2 * kNS;
  block_fx<kBlock, kNT>(acc, sh, out);
  if (threadIdx.x < 2 * (kNS - kNT)) out[2 * kNT + threadIdx.x] = 0;
}

__global__ void __launch_bounds__(kBlock) k_corr_flags(const int32_t* __restrict__ cj, int64_t ns,
                                                       uint8_t* __restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += (int64_t)gridDim.x * blockDim.x)
    flags[i] = cj[i] >= 0 ? 1 : 0;
}

__global__ void __launch_bounds__(kBlock) k_corr_pairs(const int32_t* __restrict__ cj, const int32_t* __restrict__ src_idx,
                                                       int64_t m, int32_t* __restrict__ corr) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
    int32_t i = src_idx[k];
    corr[2 * k] = i;
    corr[2 * k + 1] = cj[i];
  }
}

// ------------------------------------------------------------ host linear algebra
static bool ldlt_solve6(const double A_in[36], const double b_in[6], double x[6]) {
  double A[36];
  std::memcpy(A, A_in, sizeof(A));
  int perm[6] = {0, 1, 2, 3, 4, 5};
  const int n = 6;
  for (int k = 0; k < n; ++k) {
    int piv = k;
    double best = std::fabs(A[k * n + k]);
    for (int i = k + 1; i < n; ++i)
      if (std::fabs(A[i * n + i]) > best) {
        best = std::fabs(A[i * n + i]);
        piv = i;
      }
    if (piv != k) {
      for (int j = 0; j < n; ++j) std::swap(A[k * n + j], A[piv * n + j]);
      for (int i = 0; i < n; ++i) std::swap(A[i * n + k], A[i * n + piv]);
      std::swap(perm[k], perm[piv]);
    }
    const double dk = A[k * n + k];
    double col[6];
    for (int i = k + 1; i < n; ++i) col[i] = A[i * n + k];
    for (int i = k + 1; i < n; ++i)
      for (int j = k + 1; j < n; ++j) A[i * n + j] -= dk != 0 ? col[i] * col[j] / dk : 0.0;
    for (int i = k + 1; i < n; ++i) A[i * n + k] = dk != 0 ? col[i] / dk : 0.0;
  }
  double y[6];
  for (int i = 0; i < n; ++i) y[i] = b_in[perm[i]];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < i; ++j) y[i] -= A[i * n + j] * y[j];
  const double tiny = std::numeric_limits<double>::min();
  for (int i = 0; i < n; ++i) y[i] = std::fabs(A[i * n + i]) > tiny ? y[i] / A[i * n + i] : 0.0;
  for (int i = n - 1; i >= 0; --i)
    for (int j = i + 1; j < n; ++j) y[i] -= A[j * n + i] * y[j];
  for (int i = 0; i < n; ++i) x[perm[i]] = y[i];
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(x[i])) return false;
  return true;
}

// TransformVector6dToMatrix4d: R = Rz(x2) Ry(x1) Rx(x0), t = x[3..5]
static void vec6_to_mat4(const double x[6], double T[16]) {
  const double ca = std::cos(x[0]), sa = std::sin(x[0]);
  const double cb = std::cos(x[1]), sb = std::sin(x[1]);
  const double cg = std::cos(x[2]), sg = std::sin(x[2]);
  const double Rz[9] = {cg, -sg, 0, sg, cg, 0, 0, 0, 1};
  const double Ry[9] = {cb, 0, sb, 0, 1, 0, -sb, 0, cb};
  const double Rx[9] = {1, 0, 0, 0, ca, -sa, 0, sa, ca};
  double A[9], R[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      A[i * 3 + j] = (Rz[i * 3] * Ry[j] + Rz[i * 3 + 1] * Ry[3 + j]) + Rz[i * 3 + 2] * Ry[6 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i * 3 + j] = (A[i * 3] * Rx[j] + A[i * 3 + 1] * Rx[3 + j]) + A[i * 3 + 2] * Rx[6 + j];
  for (int i = 0; i < 16; ++i) T[i] = 0;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) T[i * 4 + j] = R[i * 3 + j];
    T[i * 4 + 3] = x[3 + i];
  }
  T[15] = 1;
}

static void mat4_mul(const double* A, const double* B, double* C) {
  double t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      t[i * 4 + j] =
          ((A[i * 4] * B[j] + A[i * 4 + 1] * B[4 + j]) + A[i * 4 + 2] * B[8 + j]) + A[i * 4 + 3] * B[12 + j];
  std::memcpy(C, t, sizeof(t));
}

static int solve_update(const double* sums, double* upd) {
  double JTJ[36], mb[6], x[6];
  int t = 0;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) {
      JTJ[a * 6 + b] = sums[t];
      JTJ[b * 6 + a] = sums[t];
      ++t;
    }
  for (int a = 0; a < 6; ++a) mb[a] = -sums[21 + a];
  if (sums[28] <= 0.0 || !ldlt_solve6(JTJ, mb, x)) {
    for (int a = 0; a < 16; ++a) upd[a] = (a % 5 == 0) ? 1.0 : 0.0;
    return 0;
  }
  vec6_to_mat4(x, upd);
  return 1;
}

// ------------------------------------------------------------ descriptors
constexpr double kDescMagic = 4242.0;

static void desc_pack(const GridBuild& G, const void* base, const float4* normals, double* d) {
  const GridView& g = G.view;
  d[0] = g.ox; d[1] = g.oy; d[2] = g.oz; d[3] = g.h; d[4] = g.inv_h; d[5] = g.slack;
  d[6] = g.nx; d[7] = g.ny; d[8] = g.nz; d[9] = (double)g.n;
  d[10] = (double)((const char*)G.pts - (const char*)base);
  d[11] = (double)((const char*)G.start - (const char*)base);
  d[12] = (double)((const char*)normals - (const char*)base);
  d[13] = kDescMagic;
  d[14] = d[15] = 0;
}

static bool desc_unpack(const double* d, const void* base, GridView* g, const float4** normals) {
  if (!d || d[13] != kDescMagic) return false;
  g->ox = (float)d[0]; g->oy = (float)d[1]; g->oz = (float)d[2]; g->h = (float)d[3]; g->inv_h = (float)d[4];
  g->slack = (float)d[5];
  g->nx = (int)d[6]; g->ny = (int)d[7]; g->nz = (int)d[8]; g->n = (int64_t)d[9];
  g->stats = search_stats_ptr();
  g->blocked = 0;
  g->bnx = g->bny = 0;
  g->pts = (const float4*)((const char*)base + (int64_t)d[10]);
  g->start = (const int32_t*)((const char*)base + (int64_t)d[11]);
  *normals = (const float4*)((const char*)base + (int64_t)d[12]);
  return true;
}

// fx exponents of the 32 sums (common.hpp) from bounds that every rank
// derives alike — the source's |x|,|y|,|z| bounds (the whole source's, on
// every rank), T and max_correspondence_distance:
//   |p|  <= Pn = |(|T| absmax + |t|)| (row bounds of T (x,y,z,1), Euclidean)
//   |J_a| <= Pn |n| (a < 3), |n_a| (a >= 3), |n| <= 1.01 (float32 unit normal)
//   |r| = |(p - vt).n| <= d |n| < max_corr |n|,  d^2 < max_corr^2
// (1.01: margin for float rounding; a looser bound only coarsens the quantum).
static void icp_fx_exps(const double absmax[3], const double* T, double max_corr, int q[kNS]) {
  double P2 = 0.0;
  for (int i = 0; i < 3; ++i) {
    const double Pi = ((std::fabs(T[4 * i]) * absmax[0] + std::fabs(T[4 * i + 1]) * absmax[1]) +
                       std::fabs(T[4 * i + 2]) * absmax[2]) + std::fabs(T[4 * i + 3]);
    P2 += Pi * Pi;
  }
  const double pn = std::sqrt(P2) * 1.01;
  double bJ[6];
  for (int a = 0; a < 6; ++a) bJ[a] = (a < 3 ? pn : 1.0) * 1.01;
  const double br = max_corr * 1.01 * 1.01;
  int k = 0;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) q[k++] = fx_exp(bJ[a] * bJ[b] * 1.01);
  for (int a = 0; a < 6; ++a) q[21 + a] = fx_exp(bJ[a] * br * 1.01);
  q[27] = fx_exp(br * br * 1.01);
  q[28] = fx_exp(1.0);
  q[29] = fx_exp(max_corr * max_corr * 1.01);
  q[30] = q[31] = 0;
}

struct AccWs {
  int64_t* partial;
  int64_t* digits;
  int32_t* cj;
  int32_t* mpos;
  uint8_t* flags;
  int32_t* src_idx;
  int32_t* scan_tmp;
  int64_t* cnt;
  char* aabb;
  double* mm;
};

// blocks of the moments pass: <= kFxLaneTerms pairs per lane
static int icp_blocks(int64_t ns) {
  const int64_t need = (ns + (int64_t)kBlock * kFxLaneTerms - 1) / ((int64_t)kBlock * kFxLaneTerms);
  return (int)std::max<int64_t>(1, std::max<int64_t>(need, std::min<int64_t>(kIcpBlocks, (ns + kBlock - 1) / kBlock)));
}

static size_t acc_carve(Arena& ar, int64_t ns, AccWs* w) {
  w->partial = ar.take<int64_t>((size_t)icp_blocks(ns) * 2 * kNS);
  w->digits = ar.take<int64_t>(2 * kNS);
  w->cj = ar.take<int32_t>(ns);
  w->mpos = ar.take<int32_t>(ns);
  w->flags = ar.take<uint8_t>(ns + 16);
  w->src_idx = ar.take<int32_t>(ns);
  w->scan_tmp = ar.take<int32_t>(compact_workspace_ints(ns));
  w->cnt = ar.take<int64_t>(2);
  w->aabb = ar.take<char>(aabb_ws_bytes(ns));
  w->mm = ar.take<double>(8);
  return ar.used;
}

__global__ void __launch_bounds__(kBlock) k_absmax4(const float4* __restrict__ p, int64_t n, unsigned int* __restrict__ out) {
  float m[3] = {0.f, 0.f, 0.f};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = p[i];
    m[0] = fmaxf(m[0], fabsf(v.x));
    m[1] = fmaxf(m[1], fabsf(v.y));
    m[2] = fmaxf(m[2], fabsf(v.z));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int a = 0; a < 3; ++a) m[a] = fmaxf(m[a], __shfl_xor(m[a], o, 64));
  // non-negative floats order as their bits: an integer max is the float max
  if ((threadIdx.x & 63) == 0)
    for (int a = 0; a < 3; ++a) atomicMax(&out[a], __float_as_uint(m[a]));
}

// |x|,|y|,|z| bounds of a source: (n,3) float32 or the (n,4) sorted form
static int source_absmax(const float* src, int64_t ns, bool sorted, AccWs& w, hipStream_t s, double out[3]) {
  if (sorted) {
    unsigned int* u = reinterpret_cast<unsigned int*>(w.mm);
    O3DX_HIP(hipMemsetAsync(u, 0, 4 * sizeof(unsigned int), s));
    hipLaunchKernelGGL(k_absmax4, dim3(grid_for(ns, kBlock, 1024)), dim3(kBlock), 0, s,
                       reinterpret_cast<const float4*>(src), ns, u);
    unsigned int b[4];
    O3DX_TRY(read_back(b, u, sizeof(b), s));
    for (int a = 0; a < 3; ++a) {
      float f;
      std::memcpy(&f, &b[a], 4);
      out[a] = f;
    }
    return 0;
  }
  double mm[6];
  O3DX_TRY(aabb_device(src, ns, w.mm, w.aabb, s));
  O3DX_TRY(read_back(mm, w.mm, sizeof(mm), s));
  for (int a = 0; a < 3; ++a) out[a] = std::max(std::fabs(mm[a]), std::fabs(mm[3 + a]));
  return 0;
}

// absmax: the source's coordinate bounds (host, 3) — the same on every rank
// of a sharded source; fx_out (nullable, host 4 x kNS): the exact sums.
static int accumulate(const float* src, int64_t ns, bool sorted, const GridView& g, const float4* tn, const double* T,
                      double radius, const double* absmax, AccWs& w, hipStream_t s, double* sums_host,
                      int64_t* fx_out, int32_t* corr_out, int64_t* ncorr) {
  Mat4 M;
  std::memcpy(M.m, T, sizeof(M.m));
  const int nb = icp_blocks(ns);
  const bool want_corr = corr_out != nullptr;
  int q[kNS];
  icp_fx_exps(absmax, T, radius, q);
  FxScales sc;
  for (int k = 0; k < kNT; ++k) sc.s[k] = fx_scale(q[k]);
  KTimer kt("icp_accumulate", s);
  if (ns > 0) {
    int32_t* cj = want_corr ? w.cj : (int32_t*)nullptr;
    const unsigned nm = grid_for(ns, kBlock, 1 << 30);
    KTimer km("icp_match", s);
    // O3DX_ICP_SHELL=1: the Chebyshev shell walk (round 1-2 form) instead of the row walk
    const bool shell = getenv("O3DX_ICP_SHELL") != nullptr;
    if (sorted && !shell)
      hipLaunchKernelGGL((k_icp_match<true, true>), dim3(nm), dim3(kBlock), 0, s, src, ns, g, M, radius, w.mpos, cj);
    else if (sorted)
      hipLaunchKernelGGL((k_icp_match<true, false>), dim3(nm), dim3(kBlock), 0, s, src, ns, g, M, radius, w.mpos, cj);
    else if (!shell)
      hipLaunchKernelGGL((k_icp_match<false, true>), dim3(nm), dim3(kBlock), 0, s, src, ns, g, M, radius, w.mpos, cj);
    else
      hipLaunchKernelGGL((k_icp_match<false, false>), dim3(nm), dim3(kBlock), 0, s, src, ns, g, M, radius, w.mpos,
                         cj);
    km.stop();
    if (sorted)
      hipLaunchKernelGGL(k_icp_moments<true>, dim3(nb), dim3(kBlock), 0, s, src, ns, g, tn, M, w.mpos, sc, w.partial);
    else
      hipLaunchKernelGGL(k_icp_moments<false>, dim3(nb), dim3(kBlock), 0, s, src, ns, g, tn, M, w.mpos, sc, w.partial);
    O3DX_TRY(reduce_columns_i64(w.partial, nb, 2 * kNS, w.digits, s));
  } else {
    O3DX_HIP(hipMemsetAsync(w.digits, 0, 2 * kNS * sizeof(int64_t), s));
  }
  kt.stop();
  if (want_corr && ns > 0) {
    hipLaunchKernelGGL(k_corr_flags, dim3(grid_for(ns, kBlock, 8192)), dim3(kBlock), 0, s, w.cj, ns, w.flags);
    O3DX_TRY(compact_flags(w.flags, ns, w.src_idx, nullptr, w.cnt, w.scan_tmp, s));
    int64_t m = 0;
    O3DX_TRY(read_back(&m, w.cnt, sizeof(int64_t), s));
    if (m > 0)
      hipLaunchKernelGGL(k_corr_pairs, dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, w.cj, w.src_idx, m,
                         corr_out);
    if (ncorr) *ncorr = m;
  } else if (ncorr) {
    *ncorr = -1;
  }
  int64_t digits[2 * kNS], fx[4 * kNS];
  O3DX_TRY(read_back(digits, w.digits, sizeof(digits), s));
  O3DX_HIP(hipGetLastError());
  fx_pack(digits, q, kNS, fx);
  fx_to_double(fx, kNS, sums_host);
  if (fx_out) std::memcpy(fx_out, fx, sizeof(fx));
  if (ncorr && !want_corr) *ncorr = (int64_t)sums_host[28];
  return 0;
}

// grid occupancy / minimum cell for the 1-NN-within-radius search
static double icp_min_h(double max_corr) {
  if (const char* e = getenv("O3DX_ICP_MINH_DIV")) return max_corr / atof(e);  // tuning override
  return max_corr / 16.0;
}
// target grid cell capacity per point: a surface occupies few of the box's
// cells, so a finer grid than the volume default keeps the candidates per
// query low (the dense start table costs 8 B per cell)
static int icp_cap_mult() {
  if (const char* e = getenv("O3DX_ICP_CAP")) return std::max(1, atoi(e));
  return 12;
}
static double icp_occ() {
  if (const char* e = getenv("O3DX_ICP_OCC")) return atof(e);
  return 2.0;
}

}  // namespace o3dx

using namespace o3dx;

extern "C" size_t o3dx_icp_target_workspace_bytes(int64_t nt) { return grid_ws_bytes(nt, icp_cap_mult()) + 1024; }

extern "C" int o3dx_icp_target_build(const float* tgt, const float* tgt_normals, int64_t nt, double max_corr,
                                     void* target_ws, size_t target_ws_bytes, double* desc, void* stream) {
  if (nt < 0 || (nt > 0 && (!tgt || !tgt_normals)) || !desc) return fail(O3DX_EINVAL, "o3dx_icp_target_build: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  if (!target_ws || target_ws_bytes < o3dx_icp_target_workspace_bytes(nt))
    return fail(O3DX_ENOMEM, "icp target workspace too small");
  GridBuild G;
  O3DX_TRY(grid_build(tgt, nt, icp_occ(), icp_min_h(max_corr), target_ws, target_ws_bytes, as_stream(stream), &G, nullptr,
                      tgt_normals, false, icp_cap_mult()));
  desc_pack(G, target_ws, G.extra, desc);
  return 0;
}

extern "C" size_t o3dx_icp_accumulate_workspace_bytes(int64_t ns) {
  Arena ar(nullptr, 0);
  AccWs w;
  return acc_carve(ar, std::max<int64_t>(ns, 1), &w) + 1024;
}

extern "C" int o3dx_icp_accumulate(const float* src, int64_t ns, int src_sorted4, const void* target_ws,
                                   const double* desc, const double* T, double max_corr, const double* src_absmax,
                                   double* sums, int64_t* fx_out, int32_t* corr_out, int64_t* ncorr, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (ns < 0 || (ns > 0 && !src) || !target_ws || !T || !sums) return fail(O3DX_EINVAL, "o3dx_icp_accumulate: bad args");
  GridView g;
  const float4* tn;
  if (!desc_unpack(desc, target_ws, &g, &tn)) return fail(O3DX_EINVAL, "invalid ICP target descriptor");
  if (!ws || ws_bytes < o3dx_icp_accumulate_workspace_bytes(ns)) return fail(O3DX_ENOMEM, "icp workspace too small");
  Arena ar(ws, ws_bytes);
  AccWs w;
  acc_carve(ar, std::max<int64_t>(ns, 1), &w);
  hipStream_t s = as_stream(stream);
  double am[3] = {0, 0, 0};
  if (src_absmax) std::memcpy(am, src_absmax, sizeof(am));
  else if (ns > 0) O3DX_TRY(source_absmax(src, ns, src_sorted4 != 0, w, s, am));
  return accumulate(src, ns, src_sorted4 != 0, g, tn, T, max_corr, am, w, s, sums, fx_out, corr_out, ncorr);
}

extern "C" size_t o3dx_spatial_sort_workspace_bytes(int64_t n) { return grid_ws_bytes(n) + 1024; }

extern "C" int o3dx_spatial_sort(const float* xyz, int64_t n, double target_occ, float* sorted4, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !sorted4))) return fail(O3DX_EINVAL, "o3dx_spatial_sort: bad args");
  if (!ws || ws_bytes < o3dx_spatial_sort_workspace_bytes(n)) return fail(O3DX_ENOMEM, "spatial_sort workspace too small");
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  GridBuild G;
  O3DX_TRY(grid_build(xyz, n, target_occ > 0 ? target_occ : 8.0, 0.0, ws, ws_bytes, s, &G, nullptr, nullptr,
                      /*blocked=*/true));
  O3DX_HIP(hipMemcpyAsync(sorted4, G.pts, (size_t)n * sizeof(float4), hipMemcpyDeviceToDevice, s));
  return 0;
}

extern "C" int o3dx_icp_solve_point_to_plane(const double* sums, double* upd) {
  if (!sums || !upd) return fail(O3DX_EINVAL, "o3dx_icp_solve_point_to_plane: bad args");
  return solve_update(sums, upd);
}

extern "C" int o3dx_icp_update(const double* sums, double* T) {
  if (!sums || !T) return fail(O3DX_EINVAL, "o3dx_icp_update: bad args");
  double upd[16];
  const int solved = solve_update(sums, upd);
  mat4_mul(upd, T, T);
  return solved;
}

extern "C" size_t o3dx_registration_icp_workspace_bytes(int64_t ns) {
  ns = std::max<int64_t>(ns, 1);
  return Arena::align((size_t)ns * sizeof(float4) + 1) +
         std::max(o3dx_icp_accumulate_workspace_bytes(ns), o3dx_spatial_sort_workspace_bytes(ns)) + 1024;
}

extern "C" int o3dx_registration_icp_point_to_plane(const float* src, int64_t ns, const float* tgt,
                                                    const float* tgt_normals, int64_t nt, double max_corr,
                                                    const double* init, int max_iteration, double rel_fit,
                                                    double rel_rmse, double* T_out, double* fitness, double* rmse,
                                                    int32_t* corr_out, int64_t* ncorr, void* target_ws,
                                                    size_t target_ws_bytes, void* ws, size_t ws_bytes, void* stream) {
  if (!T_out || !fitness || !rmse) return fail(O3DX_EINVAL, "registration_icp: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  hipStream_t s = as_stream(stream);
  double desc[16];
  O3DX_TRY(o3dx_icp_target_build(tgt, tgt_normals, nt, max_corr, target_ws, target_ws_bytes, desc, stream));
  GridView g;
  const float4* tn;
  desc_unpack(desc, target_ws, &g, &tn);
  if (!ws || ws_bytes < o3dx_registration_icp_workspace_bytes(ns)) return fail(O3DX_ENOMEM, "icp workspace too small");
  // [sorted source float4][accumulate arena | sort scratch]
  float* src4 = (float*)ws;
  char* rest = (char*)ws + Arena::align((size_t)std::max<int64_t>(ns, 1) * sizeof(float4) + 1);
  size_t rest_bytes = ws_bytes - (size_t)(rest - (char*)ws);
  if (ns > 0) O3DX_TRY(o3dx_spatial_sort(src, ns, 8.0, src4, rest, rest_bytes, stream));
  Arena ar(rest, rest_bytes);
  AccWs w;
  acc_carve(ar, std::max<int64_t>(ns, 1), &w);
  double T[16];
  if (init) std::memcpy(T, init, sizeof(T));
  else
    for (int a = 0; a < 16; ++a) T[a] = (a % 5 == 0) ? 1.0 : 0.0;
  double sums[kNS];
  double am[3] = {0, 0, 0};
  if (ns > 0) O3DX_TRY(source_absmax(src4, ns, true, w, s, am));
  auto metrics = [&](const double* sm, double& fit, double& rm) {
    double c = sm[28];
    if (c <= 0 || ns == 0) {
      fit = 0;
      rm = 0;
    } else {
      fit = c / (double)ns;
      rm = std::sqrt(sm[29] / c);
    }
  };
  O3DX_TRY(accumulate(src4, ns, true, g, tn, T, max_corr, am, w, s, sums, nullptr, nullptr, nullptr));
  double fit, rm;
  metrics(sums, fit, rm);
  for (int it = 0; it < max_iteration; ++it) {
    double upd[16];
    solve_update(sums, upd);
    mat4_mul(upd, T, T);
    const double pf = fit, pr = rm;
    const bool last = (it + 1 == max_iteration);
    O3DX_TRY(accumulate(src4, ns, true, g, tn, T, max_corr, am, w, s, sums, nullptr, last ? corr_out : nullptr, last ? ncorr : nullptr));
    metrics(sums, fit, rm);
    if (std::fabs(pf - fit) < rel_fit && std::fabs(pr - rm) < rel_rmse) {
      if (!last && corr_out) O3DX_TRY(accumulate(src4, ns, true, g, tn, T, max_corr, am, w, s, sums, nullptr, corr_out, ncorr));
      break;
    }
  }
  if (max_iteration <= 0 && corr_out) O3DX_TRY(accumulate(src4, ns, true, g, tn, T, max_corr, am, w, s, sums, nullptr, corr_out, ncorr));
  std::memcpy(T_out, T, sizeof(T));
  *fitness = fit;
  *rmse = rm;
  if (!corr_out && ncorr) *ncorr = (int64_t)sums[28];
  return 0;
}
