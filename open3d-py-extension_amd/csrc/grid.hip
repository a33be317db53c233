// grid.hip — spatial grid build, estimate_normals, batched kNN search.
//
// estimate_normals replaces o3d PointCloud.estimate_normals(param,
// fast_normal_computation=True) (reference open3dpypro/PointCloud.py:68-73,
// processors.py:243-249 CPUNormals, :267-303 TorchNormals' role).
// Per point: neighbour set (grid.hpp), Open3D's raw-moment float64 covariance
// (ComputeCovariance), FastEigen3x3 smallest eigenvector — both in float64,
// restated from Open3D geometry/EstimateNormals.cpp, utility/Eigen.cpp.
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
    int c = cx + g.nx * (cy + g.ny * cz);
    cell[i] = c;
    rank[i] = atomicAdd(&count[c], 1);
  }
}

__global__ void __launch_bounds__(kBlock) k_count_nonzero(const int32_t* __restrict__ count, int64_t nc,
                                                          unsigned long long* __restrict__ out) {
  int64_t local = 0;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x)
    local += count[c] != 0;
  local = wave_sum(local);
  if (lane_id() == 0 && local) atomicAdd(out, (unsigned long long)local);
}

__global__ void __launch_bounds__(kBlock) k_grid_scatter(const float* __restrict__ xyz, int64_t n,
                                                         const int32_t* __restrict__ cell,
                                                         const int32_t* __restrict__ rank,
                                                         const int32_t* __restrict__ start, float4* __restrict__ pts,
                                                         const float* __restrict__ extra_src,
                                                         float4* __restrict__ extra) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t pos = (int64_t)start[cell[i]] + rank[i];
    pts[pos] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], __int_as_float((int)i));
    if (extra) extra[pos] = make_float4(extra_src[3 * i], extra_src[3 * i + 1], extra_src[3 * i + 2], 0.f);
  }
}

// deterministic in-cell order: ascending original index (atomic ranks are not)
__global__ void __launch_bounds__(kBlock) k_grid_cell_sort(const int32_t* __restrict__ start, int64_t nc,
                                                           float4* __restrict__ pts, float4* __restrict__ extra) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x) {
    int s0 = start[c], s1 = start[c + 1];
    if (s1 - s0 < 2) continue;
    for (int i = s0 + 1; i < s1; ++i) {
      float4 v = pts[i];
      float4 e = extra ? extra[i] : make_float4(0, 0, 0, 0);
      int key = __float_as_int(v.w);
      int j = i - 1;
      while (j >= s0 && __float_as_int(pts[j].w) > key) {
        pts[j + 1] = pts[j];
        if (extra) extra[j + 1] = extra[j];
        --j;
      }
      pts[j + 1] = v;
      if (extra) extra[j + 1] = e;
    }
  }
}

static int64_t cap_cells(int64_t n) { return std::max<int64_t>(4 * n, 4096); }

struct GridLayout {
  size_t pts, extra, count, start, cell, rank, scan, aabb, mm, scratch, total;
};

static GridLayout grid_layout(int64_t n) {
  n = std::max<int64_t>(n, 1);
  GridLayout L;
  size_t o = 0;
  auto put = [&](size_t bytes) {
    size_t at = o;
    o += Arena::align(bytes + 1);
    return at;
  };
  int64_t cc = cap_cells(n);
  L.pts = put(n * sizeof(float4));
  L.extra = put(n * sizeof(float4));
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

size_t grid_ws_bytes(int64_t n) { return grid_layout(n).total; }

static void dims_for(const double mn[3], const double mx[3], double h, int64_t d[3]) {
  for (int a = 0; a < 3; ++a) d[a] = (int64_t)std::floor(std::max(0.0, mx[a] - mn[a]) / h) + 1;
}

int grid_build(const float* xyz, int64_t n, double target_occ, double min_h, void* ws, size_t ws_bytes,
               hipStream_t s, GridBuild* out, float4* extra_sorted, const float* extra_src) {
  GridLayout L = grid_layout(n);
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
  G.cap_cells = cap_cells(std::max<int64_t>(n, 1));
  if (!extra_sorted && extra_src) extra_sorted = (float4*)(w + L.extra);
  G.extra = extra_sorted;

  double mm[6];
  O3DX_TRY(aabb_device(xyz, n, G.mm, G.aabb_ws, s));
  O3DX_HIP(hipMemcpyAsync(mm, G.mm, 6 * sizeof(double), hipMemcpyDeviceToHost, s));
  O3DX_HIP(hipStreamSynchronize(s));
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
  if (!(h > 0) || !std::isfinite(h)) h = 1.0;
  auto fit_cap = [&](double hh) {
    int64_t d[3];
    for (int guard = 0; guard < 64; ++guard) {
      dims_for(mn, mx, hh, d);
      double cells = (double)d[0] * d[1] * d[2];
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
    // assignment error of a float32 cell computation, both sides of a face
    g.slack = (float)(32.0 * std::ldexp(1.0, -24) * (maxabs + maxext) + 1e-6 * h);
    const int64_t nc = d[0] * d[1] * d[2];
    KTimer kt_count("grid_count", s);
    O3DX_HIP(hipMemsetAsync(G.count, 0, (nc + 1) * sizeof(int32_t), s));
    if (n > 0)
      hipLaunchKernelGGL(k_grid_count, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, g, G.count,
                         G.cell, G.rank);
    if (pass == 0 && n > 64) {
      // surface-like clouds: occupied cells are far denser than the box average
      unsigned long long occ = 0;
      O3DX_HIP(hipMemsetAsync(G.scratch, 0, sizeof(int64_t), s));
      hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(nc, kBlock, 4096)), dim3(kBlock), 0, s, G.count, nc,
                         (unsigned long long*)G.scratch);
      O3DX_HIP(hipMemcpyAsync(&occ, G.scratch, sizeof(occ), hipMemcpyDeviceToHost, s));
      O3DX_HIP(hipStreamSynchronize(s));
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
    if (n > 0) {
      hipLaunchKernelGGL(k_grid_scatter, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, xyz, n, G.cell, G.rank,
                         G.start, G.pts, extra_src, extra_sorted);
      hipLaunchKernelGGL(k_grid_cell_sort, dim3(grid_for(nc, kBlock, 8192)), dim3(kBlock), 0, s, G.start, nc, G.pts,
                         extra_sorted);
    }
    O3DX_HIP(hipGetLastError());
    break;
  }
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
  // Open3D ComputeCovariance cumulant order
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

__device__ __forceinline__ void finish_normal(int cnt, const MomAcc& acc, const float* __restrict__ prior, int oi,
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
__global__ void __launch_bounds__(kBlock) k_normals_knn(GridView g, const float* __restrict__ xyz, int kneed,
                                                        int hybrid, double radius, const float* __restrict__ prior,
                                                        float* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.n) return;
  const float4 q = g.pts[s];
  const int oi = __float_as_int(q.w);
  double bd[K];
  int bi[K];
  const int cnt = knn_search_dev<K>(g, q.x, q.y, q.z, kneed, hybrid != 0, radius, bd, bi);
  MomAcc acc;
  acc.zero();
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (j < cnt) {
      const int id = bi[j];
      acc.add((double)xyz[3 * id], (double)xyz[3 * id + 1], (double)xyz[3 * id + 2]);
    }
  finish_normal(cnt, acc, prior, oi, out);
}

__global__ void __launch_bounds__(kBlock) k_normals_radius(GridView g, double radius, const float* __restrict__ prior,
                                                           float* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.n) return;
  const float4 q = g.pts[s];
  const int oi = __float_as_int(q.w);
  int cx, cy, cz;
  grid_cell(g, q.x, q.y, q.z, cx, cy, cz);
  const double m = cell_margin(g, q.x, q.y, q.z, cx, cy, cz);
  const int rmax = shell_rmax(g, cx, cy, cz);
  const double r2 = radius * radius, qx = q.x, qy = q.y, qz = q.z;
  MomAcc acc;
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
    if ((double)r * g.h + m - g.slack >= radius) break;
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
  return std::max(2.0, k / 4.0);
}

}  // namespace o3dx

using namespace o3dx;

extern "C" size_t o3dx_normals_workspace_bytes(int64_t n) { return grid_ws_bytes(n) + 1024; }

extern "C" int o3dx_estimate_normals(const float* xyz, int64_t n, int mode, int knn, double radius,
                                     const float* prior, float* out, void* ws, size_t ws_bytes, void* stream) {
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
  double min_h = (mode == O3DX_SEARCH_KNN) ? 0.0 : 0.0;
  O3DX_TRY(grid_build(xyz, n, occ_for(mode, knn), min_h, ws, ws_bytes, s, &G));
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  KTimer kt("normals_knn", s);
  if (mode == O3DX_SEARCH_RADIUS) {
    hipLaunchKernelGGL(k_normals_radius, dim3(grid), dim3(kBlock), 0, s, G.view, radius, prior, out);
  } else {
    const int kneed = (int)std::min<int64_t>(knn, n);
    O3DX_DISPATCH_K(kneed, k_normals_knn, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, kneed,
                    mode == O3DX_SEARCH_HYBRID ? 1 : 0, radius, prior, out);
  }
  O3DX_HIP(hipGetLastError());
  return 0;
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
