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

// Debug-only search statistics (o3dx_search_stats): the one place the library
// allocates device memory, and only after o3dx_set_search_stats(1).
static unsigned long long* g_stats = nullptr;
static bool g_stats_on = false;
unsigned long long* search_stats_ptr() { return g_stats_on ? g_stats : nullptr; }

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
    g.stats = search_stats_ptr();
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


// ------------------------------------------------------------- chunk plan
__device__ __forceinline__ int query_row(const GridView& g, float4 v, const Mat4d& T, int useT) {
  float x = v.x, y = v.y, z = v.z;
  if (useT) {
    const double* t = T.m;
    const double X = v.x, Y = v.y, Z = v.z;
    x = (float)(((t[0] * X + t[1] * Y) + t[2] * Z) + t[3]);
    y = (float)(((t[4] * X + t[5] * Y) + t[6] * Z) + t[7]);
    z = (float)(((t[8] * X + t[9] * Y) + t[10] * Z) + t[11]);
  }
  int cx, cy, cz;
  grid_cell(g, x, y, z, cx, cy, cz);
  return cy + g.ny * cz;
}

__global__ void __launch_bounds__(kBlock) k_row_flags(const float4* __restrict__ q, int64_t n, GridView g, Mat4d T,
                                                      int useT, uint8_t* __restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = query_row(g, q[i], T, useT);
    flags[i] = (i == 0 || r != query_row(g, q[i - 1], T, useT)) ? 1 : 0;
  }
}

__global__ void k_run_nchunks(const int32_t* __restrict__ run_start, int64_t R, int64_t n, int qcap,
                              int32_t* __restrict__ nch) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= R) return;
  const int64_t a = run_start[k], b = (k + 1 < R) ? run_start[k + 1] : n;
  nch[k] = (int32_t)((b - a + qcap - 1) / qcap);
}

__global__ void k_emit_chunks(const int32_t* __restrict__ run_start, int64_t R, int64_t n, int qcap,
                              const int32_t* __restrict__ offs, int32_t* __restrict__ chunk_starts) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= R) return;
  const int64_t a = run_start[k], b = (k + 1 < R) ? run_start[k + 1] : n;
  int32_t o = offs[k];
  for (int64_t p = a; p < b; p += qcap) chunk_starts[o++] = (int32_t)p;
  if (k == R - 1) chunk_starts[offs[R]] = (int32_t)n;
}

size_t chunk_plan_ws_bytes(int64_t n) {
  n = std::max<int64_t>(n, 1);
  return Arena::align(n + 17) + 3 * Arena::align((n + 2) * 4) + Arena::align(scan_workspace_ints(n + 1) * 4 + 1) + 1024;
}

int chunk_plan(const float4* q, int64_t n, const GridView& g, const double* T, int qcap, int32_t* chunk_starts,
               int64_t* nchunks, void* ws, size_t ws_bytes, hipStream_t s) {
  if (ws_bytes < chunk_plan_ws_bytes(n)) return fail(O3DX_ENOMEM, "chunk plan workspace too small");
  if (n == 0) {
    *nchunks = 0;
    return 0;
  }
  Arena ar(ws, ws_bytes);
  uint8_t* flags = ar.take<uint8_t>(n + 16);
  int32_t* runs = ar.take<int32_t>(n + 1);
  int32_t* nch = ar.take<int32_t>(n + 1);
  int32_t* offs = ar.take<int32_t>(n + 1);
  int32_t* tmp = ar.take<int32_t>(scan_workspace_ints(n + 1));
  int64_t* cnt = ar.take<int64_t>(2);
  Mat4d M;
  for (int i = 0; i < 16; ++i) M.m[i] = T ? T[i] : ((i % 5 == 0) ? 1.0 : 0.0);
  hipLaunchKernelGGL(k_row_flags, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, q, n, g, M, T ? 1 : 0, flags);
  O3DX_TRY(compact_flags(flags, n, runs, nullptr, cnt, tmp, s));
  int64_t R = 0;
  O3DX_HIP(hipMemcpyAsync(&R, cnt, sizeof(R), hipMemcpyDeviceToHost, s));
  O3DX_HIP(hipStreamSynchronize(s));
  hipLaunchKernelGGL(k_run_nchunks, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s, runs, R, n, qcap, nch);
  O3DX_TRY(exclusive_scan_i32(nch, offs, R, tmp, s));
  hipLaunchKernelGGL(k_emit_chunks, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s, runs, R, n, qcap, offs,
                     chunk_starts);
  int32_t total = 0;
  O3DX_HIP(hipMemcpyAsync(&total, offs + R, sizeof(total), hipMemcpyDeviceToHost, s));
  O3DX_HIP(hipStreamSynchronize(s));
  O3DX_HIP(hipGetLastError());
  *nchunks = total;
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
                                                        float* __restrict__ out, const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ list_len) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (list ? t >= *list_len : t >= g.n) return;
  const int64_t s = list ? list[t] : t;
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


// ---------------------------------------------------------------------------
// KNN normals, histogram-select form (the default KNN path).
//
// Per query (one lane), with R = the radius inside which every point has been
// scanned after shells 0..S (R = S h + m - slack):
//   pass 1  float32 d^2 of every candidate in shells 0..S; the ones inside R
//           are counted into NB bins uniform in d^2 (LDS, 16-bit counters);
//           grow S until >= k lie inside R;
//   locate  the bin b* holding the k-th distance -> [L, U);
//   pass 2  rescan: d^2 < L(1-2e) is certainly among the k nearest (appended to
//           an LDS list), d^2 in the band [L(1-2e), U(1+2e)) is a boundary
//           candidate (LDS list), the rest is certainly out — e = 2^-20 bounds
//           the float32 distance error relative to float64;
//   pass 3  the (k - #certain) nearest boundary candidates by exact float64
//           (d^2, index), i.e. the same set as the oracle / nanoflann;
//   pass 4  Open3D's float64 raw moments over the k selected, FastEigen3x3.
// No per-candidate sorted insertion: cost is ~2 scans of the 27-cell
// neighbourhood in float32 plus O(k) float64 work.  Queries the form cannot
// settle (the shell reaches the grid edge, a boundary list overflows) go to a
// list served by the exact register top-k kernel above.
constexpr int kHistBins = 16;
constexpr int kBndCap = 16;
constexpr float kRelEps = 9.5367431640625e-07f;  // 2^-20

__device__ __forceinline__ float dist2_f32(const float4 q, const float4 p) {
  const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
  return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

template <int KMAX>
__global__ void __launch_bounds__(64) k_normals_knn_hist(GridView g, int kneed, const float* __restrict__ prior,
                                                         float* __restrict__ out, const int32_t* __restrict__ in_list,
                                                         const int32_t* __restrict__ in_len,
                                                         int32_t* __restrict__ fb_list, int32_t* __restrict__ fb_len) {
  __shared__ uint32_t hist[kHistBins / 2][64];
  __shared__ int32_t sel[KMAX][64];
  __shared__ int32_t bnd[kBndCap][64];
  const int lane = threadIdx.x;
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  if (in_list ? t >= *in_len : t >= g.n) return;
  const int64_t s = in_list ? in_list[t] : t;
  const float4 q = g.pts[s];
  const int oi = __float_as_int(q.w);
  int cx, cy, cz;
  grid_cell(g, q.x, q.y, q.z, cx, cy, cz);
  const double m = cell_margin(g, q.x, q.y, q.z, cx, cy, cz);
  const int rmax = shell_rmax(g, cx, cy, cz);
  bool fb = false;
  int S = 1;
  float R2 = 0.f;
  for (;; ++S) {
    if (S >= rmax) {  // shells would cover the whole grid: leave it to the exact path
      fb = true;
      break;
    }
    const double R = (double)S * g.h + m - g.slack;
    if (R <= 0.0) continue;
#pragma unroll
    for (int b = 0; b < kHistBins / 2; ++b) hist[b][lane] = 0u;
    R2 = (float)(R * R) * (1.0f - 4.0f * kRelEps);
    const float scale = (float)kHistBins / R2;
    int total = 0;
    for_cube_rows(g, cx, cy, cz, S, [&](int p0, int p1) {
      for_points4(g, p0, p1, [&](int, const float4 v) {
        const float d2 = dist2_f32(q, v);
        if (d2 < R2) {
          const int b = min((int)(d2 * scale), kHistBins - 1);
          hist[b >> 1][lane] += (b & 1) ? 0x10000u : 1u;
          ++total;
        }
      });
    });
    if (total >= kneed) break;
  }
  if (!fb) {
    int bstar = -1, cum = 0;
#pragma unroll
    for (int b = 0; b < kHistBins; ++b) {
      const uint32_t w = hist[b >> 1][lane];
      const int c = (b & 1) ? (int)(w >> 16) : (int)(w & 0xffffu);
      if (bstar < 0 && cum + c >= kneed) bstar = b;
      cum += c;
    }
    const float bw = R2 / (float)kHistBins;
    const float Lm = (float)bstar * bw * (1.0f - 2.0f * kRelEps);
    const float Up = (bstar == kHistBins - 1 ? R2 : (float)(bstar + 1) * bw) * (1.0f + 2.0f * kRelEps);
    int nsel = 0, nb = 0;
    for_cube_rows(g, cx, cy, cz, S, [&](int p0, int p1) {
      for_points4(g, p0, p1, [&](int p, const float4 v) {
        const float d2 = dist2_f32(q, v);
        if (d2 < Lm) {
          if (nsel < KMAX) sel[nsel][lane] = p;
          ++nsel;
        } else if (d2 < Up) {
          if (nb < kBndCap) bnd[nb][lane] = p;
          ++nb;
        }
      });
    });
    if (nsel > kneed || nb > kBndCap || nsel + nb < kneed) fb = true;
    if (!fb) {
      // exact tail: the (kneed - nsel) nearest boundary candidates by (d2_f64, index)
      const double qx = q.x, qy = q.y, qz = q.z;
      for (int t = nsel; t < kneed; ++t) {
        int bj = -1, bidx = 0x7fffffff;
        double bdd = INFINITY;
        for (int j = 0; j < nb; ++j) {
          const int p = bnd[j][lane];
          if (p < 0) continue;
          const float4 v = g.pts[p];
          const double d = dist2_f64(qx, qy, qz, v);
          const int id = __float_as_int(v.w);
          if (lex_less(d, id, bdd, bidx)) {
            bdd = d;
            bidx = id;
            bj = j;
          }
        }
        sel[t][lane] = bnd[bj][lane];
        bnd[bj][lane] = -1;
      }
      MomAcc acc;
      acc.zero();
      for (int j = 0; j < kneed; ++j) {
        const float4 v = g.pts[sel[j][lane]];
        acc.add((double)v.x, (double)v.y, (double)v.z);
      }
      finish_normal(kneed, acc, prior, oi, out);
    }
  }
  if (fb) {
    const int at = atomicAdd(fb_len, 1);
    fb_list[at] = (int32_t)s;
  }
}


// ---------------------------------------------------------------------------
// KNN normals, LDS-tile form (first level of the default KNN path).
// One block = one chunk of <= kTileQ queries in one grid row; the 9-row
// neighbour box is staged into LDS (coalesced), then every query runs the
// histogram-select passes of k_normals_knn_hist over LDS-resident candidates
// (shells 0..1 only).  Queries the tile cannot settle (fewer than k points
// within the shell-1 radius, or the box overflows LDS) are appended to
// fb_list for the global-memory form.
constexpr int kTileQ = 128;
constexpr int kTilePts = 1536;
constexpr int kTileCs = 640;

template <int KMAX>
__global__ void __launch_bounds__(kTileQ) k_normals_knn_tile(GridView g, const int32_t* __restrict__ chunk_starts,
                                                             int kneed, const float* __restrict__ prior,
                                                             float* __restrict__ out, int32_t* __restrict__ fb_list,
                                                             int32_t* __restrict__ fb_len) {
  __shared__ float4 tp[kTilePts];
  __shared__ int32_t ccs[kTileCs];
  __shared__ int32_t rows[kMaxTileRows + 1];
  __shared__ int32_t rst[kMaxTileRows];
  __shared__ uint32_t hist[kHistBins / 2][kTileQ];
  __shared__ uint16_t sel[KMAX][kTileQ];
  __shared__ uint16_t bnd[kBndCap][kTileQ];
  const int tid = threadIdx.x;
  const int q0 = chunk_starts[blockIdx.x], q1 = chunk_starts[blockIdx.x + 1];
  const int64_t s = (int64_t)q0 + tid;
  const bool active = s < q1;
  // the chunk lies in one (y,z) row and is sorted by x: first/last give the box
  int ax, ay, az, bx, by, bz;
  {
    const float4 f = g.pts[q0], l = g.pts[q1 - 1];
    grid_cell(g, f.x, f.y, f.z, ax, ay, az);
    grid_cell(g, l.x, l.y, l.z, bx, by, bz);
  }
  TileBox box;
  box.x0 = max(min(ax, bx) - 1, 0);
  box.x1 = min(max(ax, bx) + 1, g.nx - 1);
  box.y0 = max(ay - 1, 0);
  box.y1 = min(ay + 1, g.ny - 1);
  box.z0 = max(az - 1, 0);
  box.z1 = min(az + 1, g.nz - 1);
  box.nxr = box.x1 - box.x0 + 1;
  box.nyr = box.y1 - box.y0 + 1;
  const int staged = stage_tile<kTileQ>(g, box, tp, kTilePts, ccs, kTileCs, rows, rst);
  if (!active) return;  // no barrier below this point
  const float4 q = g.pts[s];
  int cx, cy, cz;
  grid_cell(g, q.x, q.y, q.z, cx, cy, cz);
  bool fb = staged < 0 || cy != ay || cz != az;
  if (!fb) {
    const double R = (double)g.h + cell_margin(g, q.x, q.y, q.z, cx, cy, cz) - g.slack;
    const float R2 = (R > 0.0) ? (float)(R * R) * (1.0f - 4.0f * kRelEps) : 0.0f;
    const float scale = (float)kHistBins / fmaxf(R2, 1e-30f);
#pragma unroll
    for (int b = 0; b < kHistBins / 2; ++b) hist[b][tid] = 0u;
    int total = 0;
    for_tile_rows(box, ccs, cx, cy, cz, [&](int a, int e) {
      for (int p = a; p < e; ++p) {
        const float d2 = dist2_f32(q, tp[p]);
        if (d2 < R2) {
          const int b = min((int)(d2 * scale), kHistBins - 1);
          hist[b >> 1][tid] += (b & 1) ? 0x10000u : 1u;
          ++total;
        }
      }
    });
    fb = total < kneed;
    if (!fb) {
      int bstar = -1, cum = 0;
#pragma unroll
      for (int b = 0; b < kHistBins; ++b) {
        const uint32_t w = hist[b >> 1][tid];
        const int c = (b & 1) ? (int)(w >> 16) : (int)(w & 0xffffu);
        if (bstar < 0 && cum + c >= kneed) bstar = b;
        cum += c;
      }
      const float bw = R2 / (float)kHistBins;
      const float Lm = (float)bstar * bw * (1.0f - 2.0f * kRelEps);
      const float Up = (bstar == kHistBins - 1 ? R2 : (float)(bstar + 1) * bw) * (1.0f + 2.0f * kRelEps);
      int nsel = 0, nb = 0;
      for_tile_rows(box, ccs, cx, cy, cz, [&](int a, int e) {
        for (int p = a; p < e; ++p) {
          const float d2 = dist2_f32(q, tp[p]);
          if (d2 < Lm) {
            if (nsel < KMAX) sel[nsel][tid] = (uint16_t)p;
            ++nsel;
          } else if (d2 < Up) {
            if (nb < kBndCap) bnd[nb][tid] = (uint16_t)p;
            ++nb;
          }
        }
      });
      fb = nsel > kneed || nb > kBndCap || nsel + nb < kneed;
      if (!fb) {
        const double qx = q.x, qy = q.y, qz = q.z;
        for (int t = nsel; t < kneed; ++t) {
          int bj = 0, bidx = 0x7fffffff;
          double bdd = INFINITY;
          for (int j = 0; j < nb; ++j) {
            const int p = bnd[j][tid];
            if (p == 0xffff) continue;
            const float4 v = tp[p];
            const double d = dist2_f64(qx, qy, qz, v);
            const int id = __float_as_int(v.w);
            if (lex_less(d, id, bdd, bidx)) {
              bdd = d;
              bidx = id;
              bj = j;
            }
          }
          sel[t][tid] = bnd[bj][tid];
          bnd[bj][tid] = 0xffff;
        }
        MomAcc acc;
        acc.zero();
        for (int j = 0; j < kneed; ++j) {
          const float4 v = tp[sel[j][tid]];
          acc.add((double)v.x, (double)v.y, (double)v.z);
        }
        finish_normal(kneed, acc, prior, __float_as_int(q.w), out);
      }
    }
  }
  if (fb) {
    const int at = atomicAdd(fb_len, 1);
    fb_list[at] = (int32_t)s;
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
  if (const char* e = getenv("O3DX_GRID_OCC")) return atof(e);  // tuning override
  if (mode == O3DX_SEARCH_RADIUS) return 4.0;
  if (mode == O3DX_SEARCH_KNN) return std::max(4.0, k / 3.0);  // histogram path: shells 0..1 hold k
  return std::max(2.0, k / 4.0);
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
  unsigned long long v[4] = {0, 0, 0, 0};
  if (g_stats && hipDeviceSynchronize() == hipSuccess)
    (void)hipMemcpy(v, g_stats, sizeof(v), hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i) out[i] = (int64_t)v[i];
  return 0;
}

extern "C" size_t o3dx_normals_workspace_bytes(int64_t n) {
  n = std::max<int64_t>(n, 1);
  return grid_ws_bytes(n) + 4 * Arena::align((n + 3) * 4) + chunk_plan_ws_bytes(n) + 4096;
}

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
  const int kneed = (int)std::min<int64_t>(knn, n);
  if (mode == O3DX_SEARCH_RADIUS) {
    hipLaunchKernelGGL(k_normals_radius, dim3(grid), dim3(kBlock), 0, s, G.view, radius, prior, out);
  } else if (mode == O3DX_SEARCH_KNN && kneed >= 1 && !getenv("O3DX_NORMALS_TOPK")) {
    // LDS tiles -> global histogram-select -> exact register top-k, each level
    // serving the queries the previous one could not settle
    Arena ar((char*)ws + grid_ws_bytes(n), ws_bytes - grid_ws_bytes(n));
    int32_t* lens = ar.take<int32_t>(4);
    int32_t* list1 = ar.take<int32_t>(n);
    int32_t* list2 = ar.take<int32_t>(n);
    int32_t* chunks = ar.take<int32_t>(n + 2);
    void* pws = ar.take<char>(chunk_plan_ws_bytes(n));
    O3DX_ARENA_CHECK(ar);
    O3DX_HIP(hipMemsetAsync(lens, 0, 4 * sizeof(int32_t), s));
    const unsigned g64 = (unsigned)((n + 63) / 64);
    const bool tiles = !getenv("O3DX_NORMALS_NO_TILES");
    if (tiles) {
      int64_t nchunks = 0;
      kt.stop();
      O3DX_TRY(chunk_plan(G.view.pts, n, G.view, nullptr, kTileQ, chunks, &nchunks, pws,
                          chunk_plan_ws_bytes(n), s));
      KTimer kt2("normals_knn", s);
      if (kneed <= 32)
        hipLaunchKernelGGL(k_normals_knn_tile<32>, dim3((unsigned)nchunks), dim3(kTileQ), 0, s, G.view, chunks,
                           kneed, prior, out, list1, lens);
      else
        hipLaunchKernelGGL(k_normals_knn_tile<64>, dim3((unsigned)nchunks), dim3(kTileQ), 0, s, G.view, chunks,
                           kneed, prior, out, list1, lens);
      if (kneed <= 32)
        hipLaunchKernelGGL(k_normals_knn_hist<32>, dim3(g64), dim3(64), 0, s, G.view, kneed, prior, out, list1, lens,
                           list2, lens + 1);
      else
        hipLaunchKernelGGL(k_normals_knn_hist<64>, dim3(g64), dim3(64), 0, s, G.view, kneed, prior, out, list1, lens,
                           list2, lens + 1);
    } else {
      if (kneed <= 32)
        hipLaunchKernelGGL(k_normals_knn_hist<32>, dim3(g64), dim3(64), 0, s, G.view, kneed, prior, out,
                           (const int32_t*)nullptr, (const int32_t*)nullptr, list2, lens + 1);
      else
        hipLaunchKernelGGL(k_normals_knn_hist<64>, dim3(g64), dim3(64), 0, s, G.view, kneed, prior, out,
                           (const int32_t*)nullptr, (const int32_t*)nullptr, list2, lens + 1);
    }
    O3DX_DISPATCH_K(kneed, k_normals_knn, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, kneed, 0, radius, prior,
                    out, list2, lens + 1);
  } else {
    O3DX_DISPATCH_K(kneed, k_normals_knn, dim3(grid), dim3(kBlock), 0, s, G.view, xyz, kneed,
                    mode == O3DX_SEARCH_HYBRID ? 1 : 0, radius, prior, out, (const int32_t*)nullptr,
                    (const int32_t*)nullptr);
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
