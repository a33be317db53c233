// icp.hip — point-to-plane ICP (north-star op; no symbol in the reference,
// attached as PointCloud.registration_icp / Processors.ICP).
//
// Semantics restated from Open3D pipelines/registration/Registration.cpp
// (RegistrationICP, GetRegistrationResultAndCorrespondences with
// SearchHybrid(p, max_corr, 1)), TransformationEstimation.cpp
// (PointToPlane::ComputeTransformation), utility/Eigen.cpp (ComputeJTJandJTr,
// SolveJacobianSystemAndObtainExtrinsicMatrix, TransformVector6dToMatrix4d).
//
// One pass per iteration (k_icp_step): transform the float32 source by the
// float64 cumulative T, nearest target within max_corr (target grid), residual
// r = (vs - vt).nt, J = [vs x nt ; nt], and the 30 moments (21 JTJ + 6 JTr +
// r^2 + count + sum d^2) as exact fx integers, reduced across the wave while
// the matched target point and normal are still in registers: no second pass
// re-gathers them.  The loop itself runs on the device: k_icp_finish sums the
// block partials, forms fitness / rmse, tests convergence, solves the 6x6
// system (LDLT with diagonal pivoting) and updates T, so the host enqueues all
// iterations and waits once.  The solve is one __host__ __device__ function
// (the build has -ffp-contract=off; division and sqrt are correctly rounded on
// both sides; sin / cos are the library's own), so the host loop of a sharded
// source (distributed.py, o3dx_icp_update) reaches the same T to the bit.
#include <cfloat>
#include <vector>

#include <type_traits>
#include <utility>

#include "grid.hpp"

namespace o3dx {

constexpr int kNS = O3DX_ICP_NSUMS;  // 32 sums: 30 used
template <int C>
using IC = std::integral_constant<int, C>;
constexpr int kNT = 30;
constexpr int kIcpCopies = 128;  // copies of the digit accumulator (spread the block atomics)

#define O3DX_HD __host__ __device__

// ----------------------------------------------- float64 math, host = device
// sin and cos of x: Cody-Waite reduction by pi/2 (three-part constant, exact
// products for |x| < 2^20 pi/2) and the fdlibm kernels on [-pi/4, pi/4]
// (within an ulp or so of the correctly rounded value).  The same operations
// on the host and on the device give the same bits.
O3DX_HD inline void det_sincos(double x, double* s, double* c) {
  const double inv_pio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00, pio2_2 = 6.07710050630396597660e-11,
               pio2_3 = 2.02226624871116645580e-21;
  const double fn = rint(x * inv_pio2);
  const double r = ((x - fn * pio2_1) - fn * pio2_2) - fn * pio2_3;
  const double z = r * r, w = z * z;
  // __sin / __cos (fdlibm, musl)
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
               S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
               C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double rs = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  const double sv = r + (z * r) * (S1 + z * rs);
  const double rc = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  const double hz = 0.5 * z, wc = 1.0 - hz;
  const double cv = wc + (((1.0 - wc) - hz) + z * rc);
  const int n = (int)(((long long)fn) & 3);
  switch (n) {
    case 0: *s = sv; *c = cv; break;
    case 1: *s = cv; *c = -sv; break;
    case 2: *s = -sv; *c = -cv; break;
    default: *s = -cv; *c = sv; break;
  }
}

O3DX_HD inline bool finite_d(double v) { return v == v && v <= DBL_MAX && v >= -DBL_MAX; }

// 6x6 LDLT with diagonal pivoting.  Every loop is unrolled with constant
// indices and the pivot's row / column exchange is a per-entry select, so on
// the device A stays in registers (a dynamically indexed private array would
// live in scratch); the exchanges are exact moves, the arithmetic is the same
// operations in the same order on the host and the device.
O3DX_HD inline bool ldlt_solve6(const double A_in[36], const double b_in[6], double x[6]) {
  constexpr int n = 6;
  double A[36];
#pragma unroll
  for (int i = 0; i < 36; ++i) A[i] = A_in[i];
  int perm[6] = {0, 1, 2, 3, 4, 5};
#pragma unroll
  for (int k = 0; k < n; ++k) {
    int piv = k;
    double best = fabs(A[k * n + k]);
#pragma unroll
    for (int i = k + 1; i < n; ++i)
      if (fabs(A[i * n + i]) > best) {
        best = fabs(A[i * n + i]);
        piv = i;
      }
#pragma unroll
    for (int i = k + 1; i < n; ++i) {
      const bool sw = piv == i;
#pragma unroll
      for (int j = 0; j < n; ++j) {  // rows k and i
        const double a = A[k * n + j], c = A[i * n + j];
        A[k * n + j] = sw ? c : a;
        A[i * n + j] = sw ? a : c;
      }
#pragma unroll
      for (int r = 0; r < n; ++r) {  // columns k and i
        const double a = A[r * n + k], c = A[r * n + i];
        A[r * n + k] = sw ? c : a;
        A[r * n + i] = sw ? a : c;
      }
      const int pk = perm[k], pi = perm[i];
      perm[k] = sw ? pi : pk;
      perm[i] = sw ? pk : pi;
    }
    const double dk = A[k * n + k];
    double col[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = k + 1; i < n; ++i) col[i] = A[i * n + k];
#pragma unroll
    for (int i = k + 1; i < n; ++i)
#pragma unroll
      for (int j = k + 1; j < n; ++j) A[i * n + j] -= dk != 0 ? col[i] * col[j] / dk : 0.0;
#pragma unroll
    for (int i = k + 1; i < n; ++i) A[i * n + k] = dk != 0 ? col[i] / dk : 0.0;
  }
  double y[6];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double v = b_in[0];
#pragma unroll
    for (int t = 1; t < n; ++t) v = perm[i] == t ? b_in[t] : v;
    y[i] = v;
  }
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) y[i] -= A[i * n + j] * y[j];
#pragma unroll
  for (int i = 0; i < n; ++i) y[i] = fabs(A[i * n + i]) > DBL_MIN ? y[i] / A[i * n + i] : 0.0;
#pragma unroll
  for (int i = n - 1; i >= 0; --i)
#pragma unroll
    for (int j = i + 1; j < n; ++j) y[i] -= A[j * n + i] * y[j];
#pragma unroll
  for (int t = 0; t < n; ++t) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < n; ++i) v = perm[i] == t ? y[i] : v;
    x[t] = v;
  }
#pragma unroll
  for (int i = 0; i < n; ++i)
    if (!finite_d(x[i])) return false;
  return true;
}

// TransformVector6dToMatrix4d: R = Rz(x2) Ry(x1) Rx(x0), t = x[3..5]
O3DX_HD inline void vec6_to_mat4(const double x[6], double T[16]) {
  double sa, ca, sb, cb, sg, cg;
  det_sincos(x[0], &sa, &ca);
  det_sincos(x[1], &sb, &cb);
  det_sincos(x[2], &sg, &cg);
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

O3DX_HD inline void mat4_mul(const double* A, const double* B, double* C) {
  double t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      t[i * 4 + j] =
          ((A[i * 4] * B[j] + A[i * 4 + 1] * B[4 + j]) + A[i * 4 + 2] * B[8 + j]) + A[i * 4 + 3] * B[12 + j];
  for (int i = 0; i < 16; ++i) C[i] = t[i];
}

O3DX_HD inline int solve_update(const double* sums, double* upd) {
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

O3DX_HD inline int fx_exp_hd(double B) {
  int e = 0;
  const double b = (B > 0.0 && B <= DBL_MAX) ? fmax(B, ldexp(1.0, -900)) : 1.0;
  frexp(b, &e);
  return e - kFxBits;
}

// fx exponents of the sums (common.hpp) from bounds that every rank derives
// alike — the source's |x|,|y|,|z| bounds (the whole source's, on every rank),
// T and max_correspondence_distance:
//   |p|  <= Pn = |(|T| absmax + |t|)| (row bounds of T (x,y,z,1), Euclidean)
//   |J_a| <= Pn |n| (a < 3), |n_a| (a >= 3), |n| <= 1.01 (float32 unit normal)
//   |r| = |(p - vt).n| <= d |n| < max_corr |n|,  d^2 < max_corr^2
// (1.01: margin for float rounding; a looser bound only coarsens the quantum).
O3DX_HD inline void icp_fx_exps(const double absmax[3], const double* T, double max_corr, int q[kNS]) {
  double P2 = 0.0;
  for (int i = 0; i < 3; ++i) {
    const double Pi =
        ((fabs(T[4 * i]) * absmax[0] + fabs(T[4 * i + 1]) * absmax[1]) + fabs(T[4 * i + 2]) * absmax[2]) +
        fabs(T[4 * i + 3]);
    P2 += Pi * Pi;
  }
  const double pn = sqrt(P2) * 1.01;
  double bJ[6];
  for (int a = 0; a < 6; ++a) bJ[a] = (a < 3 ? pn : 1.0) * 1.01;
  const double br = max_corr * 1.01 * 1.01;
  int k = 0;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) q[k++] = fx_exp_hd(bJ[a] * bJ[b] * 1.01);
  for (int a = 0; a < 6; ++a) q[21 + a] = fx_exp_hd(bJ[a] * br * 1.01);
  q[27] = fx_exp_hd(br * br * 1.01);
  q[28] = fx_exp_hd(1.0);
  q[29] = fx_exp_hd(max_corr * max_corr * 1.01);
  q[30] = q[31] = 0;
}

// fx_value: common.hpp

O3DX_HD inline void icp_metrics(const double* sums, int64_t ns, double* fit, double* rm) {
  const double c = sums[28];
  if (c <= 0 || ns == 0) {
    *fit = 0;
    *rm = 0;
  } else {
    *fit = c / (double)ns;
    *rm = sqrt(sums[29] / c);
  }
}

// The device-resident state of one accumulate / registration.
struct IcpState {
  double T[16];
  double Tp[16];  // the previous step's T (the skip proof's motion bound)
  double absmax[3];
  double sums[kNS];   // the last accumulate's
  double fit, rmse;
  int32_t q[kNS];
  int32_t done;   // the loop has converged: later steps and finishes return at once
  int32_t iters;  // updates applied
  int32_t ext_on;    // the device loop: this step searches the extended ball (margins for the skip proof)
  int32_t ext_prev;  // ... and the previous one did (the margins are valid)
  int32_t wstop;     // the sharded loop: the new T leaves some rank's target window (the host refetches)
};

O3DX_HD inline void state_set_T(IcpState& st, const double* T, double max_corr) {
  for (int i = 0; i < 16; ++i) st.Tp[i] = st.T[i];
  for (int i = 0; i < 16; ++i) st.T[i] = T[i];
  icp_fx_exps(st.absmax, st.T, max_corr, st.q);
}

struct Mat4 {
  double m[16];
};

// Source point j -> (original index, float64 position under T).  SORTED: src
// is float4 (x, y, z, bits(original index)) in the compact spatial order of
// o3dx_spatial_sort, so the 64 queries of a wave probe neighbouring target
// cells; else plain (n,3) float32 in caller order.  F64 (the float64
// boundary): double4 (x, y, z, original index) of o3dx_spatial_sort_f64, or
// plain (n,3) float64.
// Eigen 4x4 * (x,y,z,1): ((T0 x + T1 y) + T2 z) + T3 per row
__device__ __forceinline__ void apply_T(const double* t, double x, double y, double z, double* px, double* py,
                                        double* pz) {
  *px = ((t[0] * x + t[1] * y) + t[2] * z) + t[3];
  *py = ((t[4] * x + t[5] * y) + t[6] * z) + t[7];
  *pz = ((t[8] * x + t[9] * y) + t[10] * z) + t[11];
}

template <bool SORTED, bool F64 = false>
__device__ __forceinline__ int64_t icp_source(const void* __restrict__ src_, int64_t j, const Mat4& T, double* px,
                                              double* py, double* pz, double* raw = nullptr) {
  double x, y, z;
  int64_t i;
  if constexpr (F64) {
    if (SORTED) {
      const double4 v = reinterpret_cast<const double4*>(src_)[j];
      x = v.x;
      y = v.y;
      z = v.z;
      i = (int64_t)v.w;
    } else {
      const double* src = reinterpret_cast<const double*>(src_);
      i = j;
      x = src[3 * i];
      y = src[3 * i + 1];
      z = src[3 * i + 2];
    }
  } else if (SORTED) {
    const float4 v = reinterpret_cast<const float4*>(src_)[j];
    x = v.x;
    y = v.y;
    z = v.z;
    i = __float_as_int(v.w);
  } else {
    const float* src = reinterpret_cast<const float*>(src_);
    i = j;
    x = src[3 * i];
    y = src[3 * i + 1];
    z = src[3 * i + 2];
  }
  if (raw) {
    raw[0] = x;
    raw[1] = y;
    raw[2] = z;
  }
  apply_T(T.m, x, y, z, px, py, pz);
  return i;
}

// ------------------------------------------------ wave transpose reduction
// 16 int64 values per lane -> lane l holds the sum over all 64 lanes of value
// (l >> 2) & 15.  Each step halves the values a lane keeps and doubles the
// lanes summed into each: pairs (i, i + 8) across the wave halves
// (v_permlane32_swap), (i, i + 4) across 16-lane rows (v_permlane16_swap),
// then DPP exchanges with lane l ^ 8 (row_ror:8), l ^ 7 (row_half_mirror),
// l ^ 1 and l ^ 2 (quad_perm).  About 80 instructions where 16 separate wave
// sums would take ~400.  EXEC must be full.
__device__ __forceinline__ int64_t join64(uint32_t lo, uint32_t hi) {
  return (int64_t)(((uint64_t)hi << 32) | (uint64_t)lo);
}
__device__ __forceinline__ int64_t swap32_add(int64_t a, int64_t b) {
  const auto r0 = __builtin_amdgcn_permlane32_swap((uint32_t)a, (uint32_t)b, false, false);
  const auto r1 = __builtin_amdgcn_permlane32_swap((uint32_t)((uint64_t)a >> 32), (uint32_t)((uint64_t)b >> 32),
                                                   false, false);
  return join64(r0[0], r1[0]) + join64(r0[1], r1[1]);
}
__device__ __forceinline__ int64_t swap16_add(int64_t a, int64_t b) {
  const auto r0 = __builtin_amdgcn_permlane16_swap((uint32_t)a, (uint32_t)b, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap((uint32_t)((uint64_t)a >> 32), (uint32_t)((uint64_t)b >> 32),
                                                   false, false);
  return join64(r0[0], r1[0]) + join64(r0[1], r1[1]);
}
template <int CTRL>
__device__ __forceinline__ int64_t dpp64(int64_t v) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)v >> 32), CTRL, 0xf, 0xf, false);
  return join64((uint32_t)lo, (uint32_t)hi);
}
// keep one of (a, b) by the lane bit, add the partner's copy of it
template <int CTRL>
__device__ __forceinline__ int64_t pair_add(int64_t a, int64_t b, bool bit) {
  return (bit ? b : a) + dpp64<CTRL>(bit ? a : b);
}

// value i = v(IC<i>): produced pair by pair as the first step consumes them
// (eight partial sums live, not sixteen values)
template <class V>
__device__ __forceinline__ int64_t wave_transpose_sum16(V&& v, int lane) {
  int64_t w[8], x[4], y[2];
  w[0] = swap32_add(v(IC<0>{}), v(IC<8>{}));  // lanes >= 32: value i + 8
  w[1] = swap32_add(v(IC<1>{}), v(IC<9>{}));
  w[2] = swap32_add(v(IC<2>{}), v(IC<10>{}));
  w[3] = swap32_add(v(IC<3>{}), v(IC<11>{}));
  w[4] = swap32_add(v(IC<4>{}), v(IC<12>{}));
  w[5] = swap32_add(v(IC<5>{}), v(IC<13>{}));
  w[6] = swap32_add(v(IC<6>{}), v(IC<14>{}));
  w[7] = swap32_add(v(IC<7>{}), v(IC<15>{}));
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = swap16_add(w[i], w[i + 4]);  // odd rows: value i + 4
#pragma unroll
  for (int i = 0; i < 2; ++i) y[i] = pair_add<0x128>(x[i], x[i + 2], (lane & 8) != 0);  // row_ror:8 = l ^ 8
  int64_t z = pair_add<0x141>(y[0], y[1], (lane & 4) != 0);  // row_half_mirror = l ^ 7
  z += dpp64<0xB1>(z);                                        // quad_perm [1,0,3,2] = l ^ 1
  z += dpp64<0x4E>(z);                                        // quad_perm [2,3,0,1] = l ^ 2
  return z;
}

// term k (Open3D ComputeJTJandJTr order: JTJ upper triangle row by row, JTr,
// r^2; then count and d^2)
constexpr int jtj_a(int k) {
  int a = 0, t = k;
  while (t >= 6 - a) {
    t -= 6 - a;
    ++a;
  }
  return a;
}
constexpr int jtj_b(int k) {
  int a = 0, t = k;
  while (t >= 6 - a) {
    t -= 6 - a;
    ++a;
  }
  return a + t;
}
// (J, r, d2 and one are all zero for a lane without a match: every term 0)
template <int K>
__device__ __forceinline__ double icp_term(const double (&J)[6], double r, double d2, double one) {
  if constexpr (K < 21) {
    constexpr int a = jtj_a(K), b = jtj_b(K);
    return J[a] * J[b];
  } else if constexpr (K < 27)
    return J[K - 21] * r;
  else if constexpr (K == 27)
    return r * r;
  else if constexpr (K == 28)
    return one;
  else
    return d2;
}
// fx_term(t, 2^-q) as ldexp then the magic add: ldexp is exact (a result
// below 2^-1022 rounds to 0 either way), so the bits equal the fma form's
__device__ __forceinline__ int64_t fx_term_q(double t, int q) {
  return (int64_t)__double_as_longlong(ldexp(t, -q) + kFxMagic) - kFxMagicBits;
}
template <int K>
__device__ __forceinline__ int64_t icp_fx(const double (&J)[6], double r, double d2, double one,
                                          const int32_t* __restrict__ q) {
  if constexpr (K >= kNT)
    return 0;
  else
    return fx_term_q(icp_term<K>(J, r, d2, one), q[K]);
}

// block b -> a bijection on [0, nb) giving XCD x = b % 8 the contiguous run
// [x q + min(x, r), ...) of the nb blocks (q = nb / 8, r = nb % 8)
__device__ __forceinline__ unsigned icp_xcd_block(unsigned b, unsigned nb) {
  const unsigned x = b & 7, i = b >> 3, q = nb >> 3, r = nb & 7;
  return x * q + min(x, r) + i;
}

// One ICP pass, a thread per source point (a full grid: the hardware balances
// the uneven searches; a loop over several batches per wave costs 25 VGPRs of
// scalar spills): the transform, the 1-NN (nn_search_dev) and, when matched,
// the 30 moment terms as fx integers (common.hpp), reduced across the wave at
// once (lane l keeps term l >> 2 of each half of 16) and split into
// {lo = low 32 bits, hi = the rest} digits; the block's digits are added
// (memory-side atomics, ~0.5 KB per block) into one of kIcpCopies accumulator
// copies (acc[copy][2 kNS]).  mpos[j]
// = the match's sorted target position (-1: none).  Integer sums: the same
// bits for any split of the source over lanes, blocks or ranks.
// round a non-negative double down to float
__device__ __forceinline__ float float_down(double x) {
  float f = (float)x;
  if ((double)f > x && f > 0.0f) f = __int_as_float(__float_as_int(f) - 1);
  return f;
}

#ifndef ICP_W2
#define ICP_W2 6
#endif
#ifndef ICP_W1
#define ICP_W1 8
#endif
// MODE 0: the plain step (accumulate); the device loop launches MODE 1 and 2
// each step, and the one the state picks runs: 1 the plain search, 2 the skip
// proof with extended-ball searches (SKIP)
// (Measured and dropped, round 6: one merged launch whose waves take the
// state's branch at run time instead of the two launches of which one returns
// at once — 2700 against 2750 it/s at C3: the merged kernel's register
// allocation costs the search steps more than the 9 us empty launch.)
template <bool SORTED, bool F64 = false, int MODE = 0>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(MODE == 2 ? ICP_W2 : ICP_W1))) k_icp_step(const void* __restrict__ src, int64_t ns, GridView g,
                                                     const float4* __restrict__ tnorm,
                                                     const IcpState* __restrict__ st, double radius,
                                                     int32_t* __restrict__ mpos, int use_prior,
                                                     int64_t* __restrict__ acc, float* __restrict__ budget,
                                                     double ext, float4* __restrict__ mca,
                                                     float2* __restrict__ mcb) {
  constexpr bool SKIP = MODE == 2;
  __shared__ int64_t sh[kBlock / 64][2 * kNS];
  if (st->done) return;  // converged: the loop's remaining steps do nothing
  if (MODE == 1 && st->ext_on) return;
  if (MODE == 2 && !st->ext_on) return;
  Mat4 T;
#pragma unroll
  for (int i = 0; i < 16; ++i) T.m[i] = st->T[i];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t alo[2] = {0, 0}, ahi[2] = {0, 0};
  {
    // workgroups are dealt round-robin over the 8 XCDs: each XCD takes a
    // contiguous run of the spatially sorted source instead, so the target
    // cells its waves probe stay in its own L2
    const int64_t j = (int64_t)icp_xcd_block(blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    int pos = -1;
    double px = 0, py = 0, pz = 0, d2 = 0, vx = 0, vy = 0, vz = 0;
    float4 nt = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < ns) {
      double raw[3];
      icp_source<SORTED, F64>(src, j, T, &px, &py, &pz, raw);
      bool kept = false;
      if (SKIP && use_prior && st->ext_prev) {
        // Skip proof: the last full search of this point left every other
        // target point at least budget[j] farther than its match (EXT below),
        // less twice each later motion.  The point moved by delta since the
        // previous step (|T p - Tp p|, from the same products the step forms),
        // so the match stays the unique nearest — the same (d^2, index) minimum
        // a full search returns — while budget > 2 delta (+ a rounding guard).
        const float b = budget[j];
        // b > 0 only after a full search matched (budget 0 otherwise), so a
        // float32 target's cached match needs no mpos read (4 B per point of
        // a skip step's 48); a float64 target gathers by position
        const int mp = F64 ? mpos[j] : 0;
        if (mp >= 0 && b > 0.0f) {
          // the match's point and normal: float32 targets read them from the
          // match cache the last full search wrote (mca / mcb, in source
          // order: coalesced, where gathers by target position are not),
          // float64 targets gather them
          double cx, cy, cz;
          float4 cn;
          if constexpr (F64) {
            const double4 c = g.pts64[mp];
            cx = c.x;
            cy = c.y;
            cz = c.z;
            cn = tnorm[mp];
          } else {
            const float4 a = mca[j];
            const float2 bb = mcb[j];
            cx = a.x;
            cy = a.y;
            cz = a.z;
            cn = make_float4(a.w, bb.x, bb.y, 0.f);
          }
          double qx, qy, qz;
          apply_T(st->Tp, raw[0], raw[1], raw[2], &qx, &qy, &qz);
          const double dx = px - qx, dy = py - qy, dz = pz - qz;
          const double guard = 1e-12 * (fabs(px) + fabs(py) + fabs(pz));
          const double left = (double)b - 2.0 * (sqrt(dx * dx + dy * dy + dz * dz) * (1.0 + 1e-12) + guard);
          // the match's exact d^2 at the new position (nanoflann order, as exact_d2)
          const double ex = px - cx, ey = py - cy, ez = pz - cz;
          double d = ex * ex;
          d = d + ey * ey;
          d = d + ez * ez;
          if (left > 0.0 && d < radius * radius) {
            kept = true;
            pos = mp;
            d2 = d;
            vx = cx;
            vy = cy;
            vz = cz;
            nt = cn;
            budget[j] = float_down(left);
          }
        }
      }
      if (!kept) {
        // the previous iteration's match as the starting bound (exact either way)
        if constexpr (SKIP) {
          double marg;
          nn_search_dev<true, F64, true>(g, px, py, pz, radius, &d2, &pos, use_prior ? mpos[j] : -1, ext, &marg);
          budget[j] = pos >= 0 ? float_down(marg) : 0.0f;
        } else {
          nn_search_dev<true, F64>(g, px, py, pz, radius, &d2, &pos, use_prior ? mpos[j] : -1);
        }
        mpos[j] = pos;
        if (pos >= 0) {
          if constexpr (F64) {
            const double4 v = g.pts64[pos];
            vx = v.x;
            vy = v.y;
            vz = v.z;
          } else {
            const float4 v = g.pts[pos];
            vx = v.x;
            vy = v.y;
            vz = v.z;
          }
          nt = tnorm[pos];
          if constexpr (SKIP && !F64) {  // the match cache of the next steps' skip proofs
            mca[j] = make_float4((float)vx, (float)vy, (float)vz, nt.x);
            mcb[j] = make_float2(nt.y, nt.z);
          }
        }
      }
    }
    const bool m = pos >= 0;
    double J[6] = {0, 0, 0, 0, 0, 0}, r = 0;
    const double one = m ? 1.0 : 0.0;
    if (!m) d2 = 0.0;
    if (m) {
    const double nx = nt.x, ny = nt.y, nz = nt.z;
      r = ((px - vx) * nx + (py - vy) * ny) + (pz - vz) * nz;
      J[0] = py * nz - pz * ny;
      J[1] = pz * nx - px * nz;
      J[2] = px * ny - py * nx;
      J[3] = nx;
      J[4] = ny;
      J[5] = nz;
    }
    const int32_t* q = st->q;
    {
      const int64_t z = wave_transpose_sum16(
          [&](auto ci) { return icp_fx<decltype(ci)::value>(J, r, d2, one, q); }, lane);
      alo[0] += z & 0xffffffffll;
      ahi[0] += z >> 32;
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      const int64_t z = wave_transpose_sum16(
          [&](auto ci) { return icp_fx<16 + decltype(ci)::value>(J, r, d2, one, q); }, lane);
      alo[1] += z & 0xffffffffll;
      ahi[1] += z >> 32;
    }
  }
  if ((lane & 3) == 0) {
    const int t = lane >> 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      sh[wv][2 * (16 * h + t)] = alo[h];
      sh[wv][2 * (16 * h + t) + 1] = ahi[h];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * kNT) {
    int64_t s = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += sh[w][threadIdx.x];
    if (s)
      atomicAdd(reinterpret_cast<unsigned long long*>(&acc[(blockIdx.x % kIcpCopies) * 2 * kNS + threadIdx.x]),
                (unsigned long long)s);
  }
}

// The digit sums of the accumulator copies (one workgroup of 1024), which are
// zeroed again for the next step; dig (LDS) receives 2 kNS digits.
__device__ __forceinline__ void collect_digits(int64_t* __restrict__ acc, int64_t (*red)[2 * kNS]) {
  const int c = threadIdx.x & 63, grp = threadIdx.x >> 6;
  int64_t a = 0;
  for (int r = grp; r < kIcpCopies; r += 16) {
    a += acc[r * 2 * kNS + c];
    acc[r * 2 * kNS + c] = 0;
  }
  red[grp][c] = a;
  __syncthreads();
  if (threadIdx.x < 2 * kNS) {
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][threadIdx.x];
    red[0][threadIdx.x] = s;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(1024) k_icp_collect(int64_t* __restrict__ acc, int64_t* __restrict__ digits) {
  __shared__ int64_t red[16][2 * kNS];
  collect_digits(acc, red);
  if (threadIdx.x < 2 * kNS) digits[threadIdx.x] = red[0][threadIdx.x];
}

// Sharded loop: whether the x-range every rank's source box can reach under T
// (+ the correspondence radius, the rounding slack and `widen`, the skip
// proof's ball extension) still lies inside that rank's target window.  win:
// world rows {box min xyz, box max xyz, window lo, window hi}; a rank without
// source rows has a non-finite box and needs nothing.  The arithmetic is
// distributed.WindowedTarget._need's, so every rank decides alike.
__device__ inline bool windows_cover(const double* __restrict__ win, int world, const double* T, double mc,
                                     double widen) {
  for (int r = 0; r < world; ++r) {
    const double* b = win + 8 * r;
    bool fin = true;
    for (int a = 0; a < 6; ++a) fin = fin && isfinite(b[a]);
    if (!fin) continue;
    double lo = INFINITY, hi = -INFINITY, am = 0.0;
    for (int c = 0; c < 8; ++c) {
      const double x = (c & 1) ? b[3] : b[0], y = (c & 2) ? b[4] : b[1], z = (c & 4) ? b[5] : b[2];
      const double xs = ((x * T[0] + y * T[1]) + z * T[2]) + T[3];
      lo = fmin(lo, xs);
      hi = fmax(hi, xs);
      am = fmax(am, fabs(xs));
    }
    const double eps = 1e-6 * (1.0 + am + mc);
    if (!(b[6] <= lo - mc - eps - widen && hi + mc + eps + widen <= b[7])) return false;
  }
  return true;
}

// The loop's per-iteration bookkeeping, one workgroup: the digit sums of the
// step's accumulator copies (or, in the sharded loop, the digits summed over
// the ranks), then (thread 0) the sums, fitness and rmse, Open3D's
// convergence test against the previous iteration's, and — while iterations
// remain — the solve and T <- update * T with the next fx exponents.
__global__ void __launch_bounds__(1024) k_icp_finish(IcpState* __restrict__ st, int64_t* __restrict__ acc,
                                                     int64_t ns, double max_corr, double rel_fit, double rel_rmse,
                                                     int it, int max_it, double ext,
                                                     const int64_t* __restrict__ digits = nullptr,
                                                     const double* __restrict__ win = nullptr, int world = 0,
                                                     double widen = 0.0) {
  __shared__ int64_t red[16][2 * kNS];
  __shared__ IcpState ls;
  __shared__ double sums[kNS];
  if (st->done) return;
  // the state into LDS by all threads at once (one thread alone would wait on
  // each global access in turn)
  constexpr int kWords = (int)(sizeof(IcpState) / sizeof(uint32_t));
  for (int t = threadIdx.x; t < kWords; t += blockDim.x)
    reinterpret_cast<uint32_t*>(&ls)[t] = reinterpret_cast<const uint32_t*>(st)[t];
  if (digits) {
    if (threadIdx.x < 2 * kNS) red[0][threadIdx.x] = digits[threadIdx.x];
    __syncthreads();
  } else {
    collect_digits(acc, red);  // (its barriers also publish ls)
  }
  if (threadIdx.x < kNS)
    sums[threadIdx.x] =
        threadIdx.x < kNT ? fx_value(red[0][2 * threadIdx.x], red[0][2 * threadIdx.x + 1], ls.q[threadIdx.x]) : 0.0;
  __syncthreads();
  if (threadIdx.x == 0) {
    double sm[kNS];
    for (int k = 0; k < kNS; ++k) sm[k] = sums[k];
    double fit, rm;
    icp_metrics(sm, ns, &fit, &rm);
    const double pf = ls.fit, pr = ls.rmse;
    for (int k = 0; k < kNS; ++k) ls.sums[k] = sm[k];
    ls.fit = fit;
    ls.rmse = rm;
    if (it > 0 && fabs(pf - fit) < rel_fit && fabs(pr - rm) < rel_rmse) {
      ls.done = 1;
    } else if (it < max_it) {
      double upd[16], T[16];
      solve_update(sm, upd);
      mat4_mul(upd, ls.T, T);
      // the update's motion bound over the source box: |(T - T_old) p| per row
      double mv = 0.0;
      for (int r = 0; r < 3; ++r) {
        const double e = fabs(T[4 * r] - ls.T[4 * r]) * ls.absmax[0] + fabs(T[4 * r + 1] - ls.T[4 * r + 1]) * ls.absmax[1] +
                         fabs(T[4 * r + 2] - ls.T[4 * r + 2]) * ls.absmax[2] + fabs(T[4 * r + 3] - ls.T[4 * r + 3]);
        mv += e * e;
      }
      state_set_T(ls, T, max_corr);
      ls.iters = it + 1;
      // the next step searches the extended ball (margins for the skip proof)
      // once the updates move the source by less than half of the extension:
      // before that the margins could not survive the next motion anyway
      ls.ext_prev = ls.ext_on;
      ls.ext_on = ext > 0.0 && sqrt(mv) < 0.5 * ext ? 1 : 0;
      if (win && !windows_cover(win, world, ls.T, max_corr, widen)) {
        ls.done = 1;  // the next step needs other target rows: the host refetches and resumes
        ls.wstop = 1;
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kWords; t += blockDim.x)
    reinterpret_cast<uint32_t*>(st)[t] = reinterpret_cast<const uint32_t*>(&ls)[t];
}

// correspondences of the last step by original source index: cj[i] = the
// target's original index, -1 for none
template <bool SORTED, bool F64 = false>
__global__ void __launch_bounds__(kBlock) k_corr_from_mpos(const void* __restrict__ src, int64_t ns, GridView g,
                                                           const int32_t* __restrict__ mpos, int32_t* __restrict__ cj) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ns; j += (int64_t)gridDim.x * blockDim.x) {
    const int pos = mpos[j];
    const int64_t i = !SORTED ? j
                      : F64   ? (int64_t)reinterpret_cast<const double4*>(src)[j].w
                              : (int64_t)__float_as_int(reinterpret_cast<const float4*>(src)[j].w);
    cj[i] = pos >= 0 ? __float_as_int(g.pts[pos].w) : -1;
  }
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

// ------------------------------------------------------------ descriptors
constexpr double kDescMagic = 4242.0;

// d[14]: offset of the float64 coordinates (float64 targets, d[15] = 1), d[16..18] their frame origin
static void desc_pack(const GridBuild& G, const void* base, const float4* normals, double* d) {
  const GridView& g = G.view;
  for (int k = 0; k < O3DX_ICP_DESC_LEN; ++k) d[k] = 0;
  d[0] = g.ox; d[1] = g.oy; d[2] = g.oz; d[3] = g.h; d[4] = g.inv_h; d[5] = g.slack;
  d[6] = g.nx; d[7] = g.ny; d[8] = g.nz; d[9] = (double)g.n;
  d[10] = (double)((const char*)G.pts - (const char*)base);
  d[11] = (double)((const char*)G.start - (const char*)base);
  d[12] = (double)((const char*)normals - (const char*)base);
  d[13] = kDescMagic;
  if (G.pts64) {
    d[14] = (double)((const char*)G.pts64 - (const char*)base);
    d[15] = 1;
    d[16] = g.o64x;
    d[17] = g.o64y;
    d[18] = g.o64z;
  }
}

static bool desc_is_f64(const double* d) { return d && d[15] == 1; }

static bool desc_unpack(const double* d, const void* base, GridView* g, const float4** normals) {
  if (!d || d[13] != kDescMagic) return false;
  *g = GridView{};
  g->ox = (float)d[0]; g->oy = (float)d[1]; g->oz = (float)d[2]; g->h = (float)d[3]; g->inv_h = (float)d[4];
  g->slack = (float)d[5];
  g->nx = (int)d[6]; g->ny = (int)d[7]; g->nz = (int)d[8]; g->n = (int64_t)d[9];
  g->stats = search_stats_ptr();
  g->blocked = 0;
  g->bnx = g->bny = 0;
  g->pts = (const float4*)((const char*)base + (int64_t)d[10]);
  g->start = (const int32_t*)((const char*)base + (int64_t)d[11]);
  *normals = (const float4*)((const char*)base + (int64_t)d[12]);
  if (desc_is_f64(d)) {
    g->pts64 = (const double4*)((const char*)base + (int64_t)d[14]);
    g->o64x = d[16];
    g->o64y = d[17];
    g->o64z = d[18];
  }
  return true;
}

struct AccWs {
  IcpState* st;
  int64_t* acc;  // [kIcpCopies][2 kNS], zero between steps
  int64_t* digits;
  int32_t* cj;
  int32_t* mpos;
  float* budget;  // the device loop's skip proof: margin left per source point
  float4* mca;    // ... and its match cache: (target x, y, z, normal x) per source point
  float2* mcb;    // (normal y, z)
  uint8_t* flags;
  int32_t* src_idx;
  int32_t* scan_tmp;
  int64_t* cnt;
  char* aabb;
  double* mm;
};

static unsigned step_blocks(int64_t ns) { return grid_for(ns, kBlock, 1ll << 31); }

static size_t acc_carve(Arena& ar, int64_t ns, AccWs* w) {
  w->st = ar.take<IcpState>(1);
  w->acc = ar.take<int64_t>((size_t)kIcpCopies * 2 * kNS);
  w->digits = ar.take<int64_t>(2 * kNS);
  w->cj = ar.take<int32_t>(ns);
  w->mpos = ar.take<int32_t>(ns);
  w->budget = ar.take<float>(ns);
  w->mca = ar.take<float4>(ns);
  w->mcb = ar.take<float2>(ns);

  w->flags = ar.take<uint8_t>(ns + 16);
  w->src_idx = ar.take<int32_t>(ns);
  w->scan_tmp = ar.take<int32_t>(compact_workspace_ints(ns));
  w->cnt = ar.take<int64_t>(2);
  // scratch of the source bounds: the float32 partials (aabb_ws_bytes) or,
  // for a float64 source, the float64 ones (aabb64_ws_bytes, twice as wide)
  w->aabb = ar.take<char>(std::max(aabb_ws_bytes(ns), aabb64_ws_bytes()));
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

__global__ void __launch_bounds__(kBlock) k_absmax_d4(const double4* __restrict__ p, int64_t n,
                                                      unsigned long long* __restrict__ out) {
  double m[3] = {0.0, 0.0, 0.0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double4 v = p[i];
    m[0] = fmax(m[0], fabs(v.x));
    m[1] = fmax(m[1], fabs(v.y));
    m[2] = fmax(m[2], fabs(v.z));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int a = 0; a < 3; ++a) m[a] = fmax(m[a], __shfl_xor(m[a], o, 64));
  // non-negative doubles order as their bits
  if ((threadIdx.x & 63) == 0)
    for (int a = 0; a < 3; ++a) atomicMax(&out[a], (unsigned long long)__double_as_longlong(m[a]));
}

// |x|,|y|,|z| bounds of a source: (n,3) float32 or the (n,4) sorted form;
// f64: (n,3) float64 or the double4 sorted form
static int source_absmax(const void* src_, int64_t ns, bool sorted, AccWs& w, hipStream_t s, double out[3],
                         bool f64 = false) {
  if (f64) {
    double mm[6];
    if (sorted) {
      unsigned long long* u = reinterpret_cast<unsigned long long*>(w.mm);
      O3DX_HIP(hipMemsetAsync(u, 0, 4 * sizeof(unsigned long long), s));
      hipLaunchKernelGGL(k_absmax_d4, dim3(grid_for(ns, kBlock, 1024)), dim3(kBlock), 0, s,
                         reinterpret_cast<const double4*>(src_), ns, u);
      unsigned long long b[4];
      O3DX_TRY(read_back(b, u, sizeof(b), s));
      for (int a = 0; a < 3; ++a) out[a] = __builtin_bit_cast(double, b[a]);
      return 0;
    }
    O3DX_TRY(aabb64_device(reinterpret_cast<const double*>(src_), ns, w.mm, w.aabb, s));
    O3DX_TRY(read_back(mm, w.mm, sizeof(mm), s));
    for (int a = 0; a < 3; ++a) out[a] = std::max(std::fabs(mm[a]), std::fabs(mm[3 + a]));
    return 0;
  }
  const float* src = reinterpret_cast<const float*>(src_);
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

// use_prior: mpos holds the previous step's matches on this source (the loop)
// a float64 target (g.pts64) takes a float64 source
// skip: the device loop's skip proof (w.budget; k_icp_step), whose full
// searches cover a tenth of a cell beyond the match for the margin (measured:
// h/16 .. h/8 within noise of each other, h/4 4 % and h/2 9 % slower at C3)
static void launch_step(const void* src, int64_t ns, bool sorted, const GridView& g, const float4* tn,
                        double radius, AccWs& w, hipStream_t s, int use_prior = 0, bool skip = false) {
  const unsigned nb = step_blocks(ns);
  const double ext = 0.1 * (double)g.h;
  KTimer km("icp_match", s);
#define O3DX_STEP(SO, F6, MO)                                                                                     \
  hipLaunchKernelGGL((k_icp_step<SO, F6, MO>), dim3(nb), dim3(kBlock), 0, s, src, ns, g, tn, w.st, radius, w.mpos, \
                     use_prior, w.acc, w.budget, ext, w.mca, w.mcb)
#define O3DX_STEPS(MO)                         \
  do {                                         \
    if (f64 && sorted) O3DX_STEP(true, true, MO);   \
    else if (f64) O3DX_STEP(false, true, MO);       \
    else if (sorted) O3DX_STEP(true, false, MO);    \
    else O3DX_STEP(false, false, MO);               \
  } while (0)
  const bool f64 = g.pts64 != nullptr;
  if (skip) {  // the state picks one of the two at run time
    O3DX_STEPS(1);
    O3DX_STEPS(2);
  } else {
    O3DX_STEPS(0);
  }
#undef O3DX_STEPS
#undef O3DX_STEP
}
// correspondences of the last step into corr_out (pairs by original index)
static int corr_of_last_step(const void* src, int64_t ns, bool sorted, const GridView& g, AccWs& w, hipStream_t s,
                             int32_t* corr_out, int64_t* ncorr) {
  if (ns == 0) {
    if (ncorr) *ncorr = 0;
    return 0;
  }
  if (sorted && g.pts64)
    hipLaunchKernelGGL((k_corr_from_mpos<true, true>), dim3(grid_for(ns, kBlock, 8192)), dim3(kBlock), 0, s, src, ns, g,
                       w.mpos, w.cj);
  else if (sorted)
    hipLaunchKernelGGL(k_corr_from_mpos<true>, dim3(grid_for(ns, kBlock, 8192)), dim3(kBlock), 0, s, src, ns, g,
                       w.mpos, w.cj);
  else
    hipLaunchKernelGGL(k_corr_from_mpos<false>, dim3(grid_for(ns, kBlock, 8192)), dim3(kBlock), 0, s, src, ns, g,
                       w.mpos, w.cj);
  hipLaunchKernelGGL(k_corr_flags, dim3(grid_for(ns, kBlock, 8192)), dim3(kBlock), 0, s, w.cj, ns, w.flags);
  O3DX_TRY(compact_flags(w.flags, ns, w.src_idx, nullptr, w.cnt, w.scan_tmp, s));
  int64_t m = 0;
  O3DX_TRY(read_back(&m, w.cnt, sizeof(int64_t), s));
  if (m > 0)
    hipLaunchKernelGGL(k_corr_pairs, dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, w.cj, w.src_idx, m,
                       corr_out);
  if (ncorr) *ncorr = m;
  return 0;
}

// One accumulate with T on the host (the sharded loop of distributed.py):
// absmax: the source's coordinate bounds (host, 3) — the same on every rank
// of a sharded source; fx_out (nullable, host 4 x kNS): the exact sums.
static int accumulate(const void* src, int64_t ns, bool sorted, const GridView& g, const float4* tn, const double* T,
                      double radius, const double* absmax, AccWs& w, hipStream_t s, double* sums_host,
                      int64_t* fx_out, int32_t* corr_out, int64_t* ncorr) {
  IcpState hs{};
  for (int a = 0; a < 3; ++a) hs.absmax[a] = absmax[a];
  state_set_T(hs, T, radius);
  KTimer kt("icp_accumulate", s);
  if (ns > 0) {
    O3DX_HIP(hipMemcpyAsync(w.st, &hs, sizeof(IcpState), hipMemcpyHostToDevice, s));
    O3DX_HIP(hipMemsetAsync(w.acc, 0, (size_t)kIcpCopies * 2 * kNS * sizeof(int64_t), s));
    launch_step(src, ns, sorted, g, tn, radius, w, s);
    hipLaunchKernelGGL(k_icp_collect, dim3(1), dim3(1024), 0, s, w.acc, w.digits);
  } else {
    O3DX_HIP(hipMemsetAsync(w.digits, 0, 2 * kNS * sizeof(int64_t), s));
  }
  kt.stop();
  if (corr_out) O3DX_TRY(corr_of_last_step(src, ns, sorted, g, w, s, corr_out, ncorr));
  else if (ncorr) *ncorr = -1;
  int64_t digits[2 * kNS], fx[4 * kNS];
  O3DX_TRY(read_back(digits, w.digits, sizeof(digits), s));
  O3DX_HIP(hipGetLastError());
  fx_pack(digits, hs.q, kNS, fx);
  for (int k = 0; k < kNS; ++k) sums_host[k] = k < kNT ? fx_value(digits[2 * k], digits[2 * k + 1], hs.q[k]) : 0.0;
  if (fx_out) std::memcpy(fx_out, fx, sizeof(fx));
  if (ncorr && !corr_out) *ncorr = (int64_t)sums_host[28];
  return 0;
}

// grid occupancy / minimum cell for the 1-NN-within-radius search (round 2
// sweeps: max_corr / 20, / 24, / 32 within +-3 % of / 16)
static double icp_min_h(double max_corr) { return max_corr / 16.0; }
// target grid cell capacity per point: a surface occupies few of the box's
// cells, so a finer grid than the volume default keeps the candidates per
// query low (the dense start table costs 8 B per cell)
static int icp_cap_mult() { return 12; }
static double icp_occ() { return 2.0; }

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
  if (desc_is_f64(desc)) return fail(O3DX_EINVAL, "a float64 ICP target takes a float64 source (o3dx_icp_register_f64)");
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

extern "C" int o3dx_spatial_sort_bounds(const float* xyz, int64_t n, double target_occ, float* sorted4,
                                        double* absmax, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !sorted4))) return fail(O3DX_EINVAL, "o3dx_spatial_sort: bad args");
  if (!ws || ws_bytes < o3dx_spatial_sort_workspace_bytes(n)) return fail(O3DX_ENOMEM, "spatial_sort workspace too small");
  if (n == 0) {
    if (absmax) absmax[0] = absmax[1] = absmax[2] = 0.0;
    return 0;
  }
  hipStream_t s = as_stream(stream);
  GridBuild G;
  O3DX_TRY(grid_build(xyz, n, target_occ > 0 ? target_occ : 8.0, 0.0, ws, ws_bytes, s, &G, nullptr, nullptr,
                      /*blocked=*/true));
  O3DX_HIP(hipMemcpyAsync(sorted4, G.pts, (size_t)n * sizeof(float4), hipMemcpyDeviceToDevice, s));
  // the exact float32 min / max, widened to double: max(|min|, |max|) per
  // axis is the largest |coordinate|, bit for bit what k_absmax4 finds
  if (absmax)
    for (int a = 0; a < 3; ++a) absmax[a] = std::max(std::fabs(G.mm_host[a]), std::fabs(G.mm_host[3 + a]));
  return 0;
}

extern "C" int o3dx_spatial_sort(const float* xyz, int64_t n, double target_occ, float* sorted4, void* ws,
                                 size_t ws_bytes, void* stream) {
  return o3dx_spatial_sort_bounds(xyz, n, target_occ, sorted4, nullptr, ws, ws_bytes, stream);
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

// The whole loop on the device: every iteration's step and finish are queued
// at once (a converged loop's remaining launches return at their first
// instruction); the host waits once for the final state.
static int run_loop(const void* src, int64_t ns, bool sorted, const GridView& g, const float4* tn, double max_corr, const double* init, int max_iteration, double rel_fit,
                    double rel_rmse, const double* absmax, AccWs& w, hipStream_t s, double* T_out, double* fitness,
                    double* rmse, int32_t* corr_out, int64_t* ncorr) {
  IcpState hs{};
  double T0[16];
  if (init) std::memcpy(T0, init, sizeof(T0));
  else
    for (int a = 0; a < 16; ++a) T0[a] = (a % 5 == 0) ? 1.0 : 0.0;
  if (ns == 0) {  // no correspondences: T unchanged, fitness and rmse 0
    std::memcpy(T_out, T0, sizeof(T0));
    *fitness = 0;
    *rmse = 0;
    if (ncorr) *ncorr = 0;
    return 0;
  }
  if (absmax) std::memcpy(hs.absmax, absmax, sizeof(hs.absmax));
  else O3DX_TRY(source_absmax(src, ns, sorted, w, s, hs.absmax, g.pts64 != nullptr));
  state_set_T(hs, T0, max_corr);
  O3DX_HIP(hipMemcpyAsync(w.st, &hs, sizeof(IcpState), hipMemcpyHostToDevice, s));
  O3DX_HIP(hipMemsetAsync(w.acc, 0, (size_t)kIcpCopies * 2 * kNS * sizeof(int64_t), s));
  const int iters = std::max(max_iteration, 0);
  // O3DX_ICP_SKIP=0 (tests, A/B): every step searches in full
  const bool skip = !(getenv("O3DX_ICP_SKIP") && atoi(getenv("O3DX_ICP_SKIP")) == 0);
  {
    KTimer kt("icp_loop", s);
    for (int it = 0; it <= iters; ++it) {
      // from the second step on, the previous step's matches seed the search
      launch_step(src, ns, sorted, g, tn, max_corr, w, s, it > 0, skip);
      hipLaunchKernelGGL(k_icp_finish, dim3(1), dim3(1024), 0, s, w.st, w.acc, ns, max_corr, rel_fit, rel_rmse, it,
                         iters, skip ? 0.1 * (double)g.h : 0.0);
    }
  }
  O3DX_HIP(hipGetLastError());
  if (corr_out) O3DX_TRY(corr_of_last_step(src, ns, sorted, g, w, s, corr_out, ncorr));
  O3DX_TRY(read_back(&hs, w.st, sizeof(IcpState), s));
  std::memcpy(T_out, hs.T, sizeof(hs.T));
  *fitness = hs.fit;
  *rmse = hs.rmse;
  if (!corr_out && ncorr) *ncorr = (int64_t)hs.sums[28];
  return 0;
}

extern "C" int o3dx_icp_register(const float* src, int64_t ns, int src_sorted4, const void* target_ws,
                                 const double* desc, const double* init, int max_iteration, double rel_fit,
                                 double rel_rmse, double max_corr, const double* src_absmax, double* T_out,
                                 double* fitness, double* rmse, int32_t* corr_out, int64_t* ncorr, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (ns < 0 || (ns > 0 && !src) || !target_ws || !T_out || !fitness || !rmse)
    return fail(O3DX_EINVAL, "o3dx_icp_register: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  if (desc_is_f64(desc)) return fail(O3DX_EINVAL, "a float64 ICP target takes a float64 source (o3dx_icp_register_f64)");
  GridView g;
  const float4* tn;
  if (!desc_unpack(desc, target_ws, &g, &tn)) return fail(O3DX_EINVAL, "invalid ICP target descriptor");
  if (!ws || ws_bytes < o3dx_icp_accumulate_workspace_bytes(ns)) return fail(O3DX_ENOMEM, "icp workspace too small");
  Arena ar(ws, ws_bytes);
  AccWs w;
  acc_carve(ar, std::max<int64_t>(ns, 1), &w);
  return run_loop(src, ns, src_sorted4 != 0, g, tn, max_corr, init, max_iteration, rel_fit, rel_rmse, src_absmax,
                  w, as_stream(stream), T_out, fitness, rmse, corr_out, ncorr);
}

// ------------------------------------------------ the sharded device loop
// distributed.registration_icp_sharded: every rank holds a share of the
// source (and the target, or the window of it its share can reach) and queues
// per iteration, with no host wait:
//   o3dx_icp_shard_step    its rows' fused match + fx-moment step (the device
//                          loop's, skip proof included) and the digit sums
//                          into digits_dev (2 x 32 int64);
//   (the caller)           a SUM all-reduce of digits_dev over the ranks (RCCL);
//   o3dx_icp_shard_finish  the loop's finish on the summed digits: sums,
//                          fitness / rmse over the GLOBAL source count, the
//                          convergence test, solve and update — the same on
//                          every rank, so every rank holds the same T.
// The fx quanta come from the global source bounds (begin's absmax), so the
// digits add exactly and T equals the single-GPU o3dx_icp_register's to the
// bit.  With windows (win_dev), the finish also stops the loop (state wstop)
// when the new T needs target rows outside some rank's window; the host reads
// the state (o3dx_icp_shard_state), refetches and calls o3dx_icp_shard_resume.
static int shard_ws(void* ws, size_t ws_bytes, int64_t ns, AccWs* w) {
  if (!ws || ws_bytes < o3dx_icp_accumulate_workspace_bytes(ns)) return fail(O3DX_ENOMEM, "icp workspace too small");
  Arena ar(ws, ws_bytes);
  acc_carve(ar, std::max<int64_t>(ns, 1), w);
  return 0;
}

extern "C" int o3dx_icp_shard_begin(const double* init, const double* src_absmax, double max_corr, int64_t ns,
                                    void* ws, size_t ws_bytes, void* stream) {
  if (ns < 0 || !src_absmax) return fail(O3DX_EINVAL, "o3dx_icp_shard_begin: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  AccWs w;
  O3DX_TRY(shard_ws(ws, ws_bytes, ns, &w));
  hipStream_t s = as_stream(stream);
  IcpState hs{};
  double T0[16];
  if (init) std::memcpy(T0, init, sizeof(T0));
  else
    for (int a = 0; a < 16; ++a) T0[a] = (a % 5 == 0) ? 1.0 : 0.0;
  std::memcpy(hs.absmax, src_absmax, sizeof(hs.absmax));
  state_set_T(hs, T0, max_corr);
  O3DX_HIP(hipMemcpyAsync(w.st, &hs, sizeof(IcpState), hipMemcpyHostToDevice, s));
  O3DX_HIP(hipMemsetAsync(w.acc, 0, (size_t)kIcpCopies * 2 * kNS * sizeof(int64_t), s));
  return 0;
}

static bool icp_skip_on() { return !(getenv("O3DX_ICP_SKIP") && atoi(getenv("O3DX_ICP_SKIP")) == 0); }

// widen: the largest skip-proof extension a window covers (the ball of a full
// search reaches 0.1 h beyond the match); a grid whose extension is larger
// searches without the skip proof.  +inf for a replicated target.
extern "C" int o3dx_icp_shard_step(const float* src, int64_t ns, int src_sorted4, const void* target_ws,
                                   const double* desc, double max_corr, int use_prior, double widen,
                                   int64_t* digits_dev, void* ws, size_t ws_bytes, void* stream) {
  if (ns < 0 || (ns > 0 && !src) || !digits_dev) return fail(O3DX_EINVAL, "o3dx_icp_shard_step: bad args");
  AccWs w;
  O3DX_TRY(shard_ws(ws, ws_bytes, ns, &w));
  hipStream_t s = as_stream(stream);
  if (ns == 0 || !target_ws) {  // nothing to match here: this rank adds zeros
    O3DX_HIP(hipMemsetAsync(digits_dev, 0, 2 * kNS * sizeof(int64_t), s));
    return 0;
  }
  if (desc_is_f64(desc)) return fail(O3DX_EINVAL, "o3dx_icp_shard_step: float32 targets only");
  GridView g;
  const float4* tn;
  if (!desc_unpack(desc, target_ws, &g, &tn)) return fail(O3DX_EINVAL, "invalid ICP target descriptor");
  launch_step(src, ns, src_sorted4 != 0, g, tn, max_corr, w, s, use_prior ? 1 : 0,
              icp_skip_on() && 0.1 * (double)g.h <= widen);
  hipLaunchKernelGGL(k_icp_collect, dim3(1), dim3(1024), 0, s, w.acc, digits_dev);
  O3DX_HIP(hipGetLastError());
  return 0;
}

extern "C" int o3dx_icp_shard_finish(const int64_t* digits_dev, int64_t n_total, int it, int max_iteration,
                                     double rel_fit, double rel_rmse, double max_corr, const double* desc,
                                     const double* win_dev, int world, double widen, int64_t ns, void* ws,
                                     size_t ws_bytes, void* stream) {
  if (!digits_dev || n_total < 0 || it < 0 || (win_dev && world < 1)) return fail(O3DX_EINVAL, "o3dx_icp_shard_finish: bad args");
  AccWs w;
  O3DX_TRY(shard_ws(ws, ws_bytes, ns, &w));
  // the skip proof's extension of this rank's target grid (0: no target here)
  const double ext =
      (desc && desc[13] == kDescMagic && icp_skip_on() && 0.1 * (double)(float)desc[3] <= widen) ? 0.1 * (double)(float)desc[3] : 0.0;
  hipLaunchKernelGGL(k_icp_finish, dim3(1), dim3(1024), 0, as_stream(stream), w.st, w.acc, std::max<int64_t>(n_total, 1),
                     max_corr, rel_fit, rel_rmse, it, std::max(max_iteration, 0), ext, digits_dev, win_dev, world,
                     widen);
  O3DX_HIP(hipGetLastError());
  return 0;
}

// info: {done, iterations applied, window stop}
extern "C" int o3dx_icp_shard_state(int64_t ns, void* ws, size_t ws_bytes, double* T_out, double* fitness,
                                    double* rmse, int32_t* info, void* stream) {
  if (!T_out || !fitness || !rmse || !info) return fail(O3DX_EINVAL, "o3dx_icp_shard_state: bad args");
  AccWs w;
  O3DX_TRY(shard_ws(ws, ws_bytes, ns, &w));
  IcpState hs;
  O3DX_TRY(read_back(&hs, w.st, sizeof(IcpState), as_stream(stream)));
  std::memcpy(T_out, hs.T, sizeof(hs.T));
  *fitness = hs.fit;
  *rmse = hs.rmse;
  info[0] = hs.done;
  info[1] = hs.iters;
  info[2] = hs.wstop;
  return 0;
}

// after a window stop: the loop continues (the host has refetched the windows;
// the next step must not reuse the previous matches: pass use_prior = 0)
extern "C" int o3dx_icp_shard_resume(int64_t ns, void* ws, size_t ws_bytes, void* stream) {
  AccWs w;
  O3DX_TRY(shard_ws(ws, ws_bytes, ns, &w));
  hipStream_t s = as_stream(stream);
  IcpState hs;
  O3DX_TRY(read_back(&hs, w.st, sizeof(IcpState), s));
  hs.done = 0;
  hs.wstop = 0;
  hs.ext_prev = 0;  // the margins were measured against the old window
  O3DX_HIP(hipMemcpyAsync(w.st, &hs, sizeof(IcpState), hipMemcpyHostToDevice, s));
  return 0;
}

extern "C" int o3dx_registration_icp_point_to_plane(const float* src, int64_t ns, const float* tgt,
                                                    const float* tgt_normals, int64_t nt, double max_corr,
                                                    const double* init, int max_iteration, double rel_fit,
                                                    double rel_rmse, double* T_out, double* fitness, double* rmse,
                                                    int32_t* corr_out, int64_t* ncorr, void* target_ws,
                                                    size_t target_ws_bytes, void* ws, size_t ws_bytes, void* stream) {
  if (!T_out || !fitness || !rmse) return fail(O3DX_EINVAL, "registration_icp: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  if (ns < 0 || (ns > 0 && !src)) return fail(O3DX_EINVAL, "registration_icp: bad args");
  hipStream_t s = as_stream(stream);
  double desc[O3DX_ICP_DESC_LEN];
  O3DX_TRY(o3dx_icp_target_build(tgt, tgt_normals, nt, max_corr, target_ws, target_ws_bytes, desc, stream));
  GridView g;
  const float4* tn;
  desc_unpack(desc, target_ws, &g, &tn);
  if (!ws || ws_bytes < o3dx_registration_icp_workspace_bytes(ns)) return fail(O3DX_ENOMEM, "icp workspace too small");
  // [sorted source float4][accumulate arena | sort scratch]
  float* src4 = (float*)ws;
  char* rest = (char*)ws + Arena::align((size_t)std::max<int64_t>(ns, 1) * sizeof(float4) + 1);
  size_t rest_bytes = ws_bytes - (size_t)(rest - (char*)ws);
  double am[3] = {0, 0, 0};
  if (ns > 0) O3DX_TRY(o3dx_spatial_sort_bounds(src, ns, 8.0, src4, am, rest, rest_bytes, stream));
  Arena ar(rest, rest_bytes);
  AccWs w;
  acc_carve(ar, std::max<int64_t>(ns, 1), &w);
  return run_loop(src4, ns, true, g, tn, max_corr, init, max_iteration, rel_fit, rel_rmse, am, w, s, T_out,
                  fitness, rmse, corr_out, ncorr);
}

// ------------------------------------------------------ float64 boundary
// point-to-plane ICP on float64 clouds (the float64 boundary, include/o3dx.h):
// the target grid is a float64 grid (grid64_build: float32 frame p - o for the
// search, exact coordinates alongside), the source is transformed from its
// float64 coordinates, and every correspondence distance, residual and
// Jacobian comes from the float64 values — Open3D's arithmetic on its
// float64 storage.  Normals stay float32 (the library's normals output).
extern "C" size_t o3dx_icp_target_f64_workspace_bytes(int64_t nt) {
  return grid64_ws_bytes(nt, icp_cap_mult()) + 1024;
}

extern "C" int o3dx_icp_target_build_f64(const double* tgt, const float* tgt_normals, int64_t nt, double max_corr,
                                         void* target_ws, size_t target_ws_bytes, double* desc, void* stream) {
  if (nt < 0 || (nt > 0 && (!tgt || !tgt_normals)) || !desc)
    return fail(O3DX_EINVAL, "o3dx_icp_target_build_f64: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  if (!target_ws || target_ws_bytes < o3dx_icp_target_f64_workspace_bytes(nt))
    return fail(O3DX_ENOMEM, "icp target workspace too small");
  GridBuild G;
  O3DX_TRY(grid64_build(tgt, nt, icp_occ(), icp_min_h(max_corr), target_ws, target_ws_bytes, as_stream(stream), &G,
                        tgt_normals, icp_cap_mult()));
  desc_pack(G, target_ws, G.extra, desc);
  return 0;
}

extern "C" size_t o3dx_spatial_sort_f64_workspace_bytes(int64_t n) { return grid64_ws_bytes(n) + 1024; }

// (n, 4) float64 copy of the cloud in o3dx_spatial_sort's order: (x, y, z,
// original index)
extern "C" int o3dx_spatial_sort_f64(const double* xyz, int64_t n, double target_occ, double* sorted4, void* ws,
                                     size_t ws_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !sorted4))) return fail(O3DX_EINVAL, "o3dx_spatial_sort_f64: bad args");
  if (!ws || ws_bytes < o3dx_spatial_sort_f64_workspace_bytes(n))
    return fail(O3DX_ENOMEM, "spatial_sort workspace too small");
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  GridBuild G;
  O3DX_TRY(grid64_build(xyz, n, target_occ > 0 ? target_occ : 8.0, 0.0, ws, ws_bytes, s, &G, nullptr, 4,
                        /*blocked=*/true));
  O3DX_HIP(hipMemcpyAsync(sorted4, G.pts64, (size_t)n * sizeof(double4), hipMemcpyDeviceToDevice, s));
  return 0;
}

extern "C" int o3dx_icp_register_f64(const double* src, int64_t ns, int src_sorted4, const void* target_ws,
                                     const double* desc, const double* init, int max_iteration, double rel_fit,
                                     double rel_rmse, double max_corr, const double* src_absmax, double* T_out,
                                     double* fitness, double* rmse, int32_t* corr_out, int64_t* ncorr, void* ws,
                                     size_t ws_bytes, void* stream) {
  if (ns < 0 || (ns > 0 && !src) || !target_ws || !T_out || !fitness || !rmse)
    return fail(O3DX_EINVAL, "o3dx_icp_register_f64: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  if (!desc_is_f64(desc)) return fail(O3DX_EINVAL, "o3dx_icp_register_f64 needs a float64 target (o3dx_icp_target_build_f64)");
  GridView g;
  const float4* tn;
  if (!desc_unpack(desc, target_ws, &g, &tn)) return fail(O3DX_EINVAL, "invalid ICP target descriptor");
  if (!ws || ws_bytes < o3dx_icp_accumulate_workspace_bytes(ns)) return fail(O3DX_ENOMEM, "icp workspace too small");
  Arena ar(ws, ws_bytes);
  AccWs w;
  acc_carve(ar, std::max<int64_t>(ns, 1), &w);
  return run_loop(src, ns, src_sorted4 != 0, g, tn, max_corr, init, max_iteration, rel_fit, rel_rmse, src_absmax,
                  w, as_stream(stream), T_out, fitness, rmse, corr_out, ncorr);
}

extern "C" size_t o3dx_registration_icp_f64_workspace_bytes(int64_t ns) {
  ns = std::max<int64_t>(ns, 1);
  return Arena::align((size_t)ns * sizeof(double4) + 1) +
         std::max(o3dx_icp_accumulate_workspace_bytes(ns), o3dx_spatial_sort_f64_workspace_bytes(ns)) + 1024;
}

extern "C" int o3dx_registration_icp_point_to_plane_f64(const double* src, int64_t ns, const double* tgt,
                                                        const float* tgt_normals, int64_t nt, double max_corr,
                                                        const double* init, int max_iteration, double rel_fit,
                                                        double rel_rmse, double* T_out, double* fitness, double* rmse,
                                                        int32_t* corr_out, int64_t* ncorr, void* target_ws,
                                                        size_t target_ws_bytes, void* ws, size_t ws_bytes,
                                                        void* stream) {
  if (!T_out || !fitness || !rmse) return fail(O3DX_EINVAL, "registration_icp_f64: bad args");
  if (!(max_corr > 0.0)) return fail(O3DX_EINVAL, "max_correspondence_distance must be > 0");
  if (ns < 0 || (ns > 0 && !src)) return fail(O3DX_EINVAL, "registration_icp_f64: bad args");
  hipStream_t s = as_stream(stream);
  double desc[O3DX_ICP_DESC_LEN];
  O3DX_TRY(o3dx_icp_target_build_f64(tgt, tgt_normals, nt, max_corr, target_ws, target_ws_bytes, desc, stream));
  GridView g;
  const float4* tn;
  desc_unpack(desc, target_ws, &g, &tn);
  if (!ws || ws_bytes < o3dx_registration_icp_f64_workspace_bytes(ns)) return fail(O3DX_ENOMEM, "icp workspace too small");
  double* src4 = (double*)ws;
  char* rest = (char*)ws + Arena::align((size_t)std::max<int64_t>(ns, 1) * sizeof(double4) + 1);
  size_t rest_bytes = ws_bytes - (size_t)(rest - (char*)ws);
  if (ns > 0) O3DX_TRY(o3dx_spatial_sort_f64(src, ns, 8.0, src4, rest, rest_bytes, stream));
  Arena ar(rest, rest_bytes);
  AccWs w;
  acc_carve(ar, std::max<int64_t>(ns, 1), &w);
  return run_loop(src4, ns, true, g, tn, max_corr, init, max_iteration, rel_fit, rel_rmse, nullptr, w, s, T_out,
                  fitness, rmse, corr_out, ncorr);
}
