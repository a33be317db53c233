// grid.hpp — uniform spatial grid over a point set (counting-sorted by cell)
// and the exact shell-expanding neighbour search used by estimate_normals,
// batched kNN search and ICP correspondences.
//
// It stands in for KDTreeFlann (nanoflann) behind o3d PointCloud.estimate_normals
// and KDTreeFlann.search_* (reference open3dpypro/PointCloud.py:68-73, :148-163):
// the neighbour *sets* are identical (exact search, float64 distances computed
// in nanoflann's order), ties at the k-th distance broken by lower index.
#pragma once

#include "common.hpp"

namespace o3dx {

struct GridView {
  const float4* __restrict__ pts;      // sorted by cell: (x, y, z, bits(original index))
  const int32_t* __restrict__ start;   // ncells + 1
  float ox, oy, oz, h, inv_h;
  float slack;                         // conservative rounding margin for the stop test
  int nx, ny, nz;
  int64_t n;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ void grid_cell(const GridView& g, float x, float y, float z, int& cx, int& cy,
                                          int& cz) {
  cx = clampi((int)floorf((x - g.ox) * g.inv_h), 0, g.nx - 1);
  cy = clampi((int)floorf((y - g.oy) * g.inv_h), 0, g.ny - 1);
  cz = clampi((int)floorf((z - g.oz) * g.inv_h), 0, g.nz - 1);
}

// signed distance from q to the faces of its (clamped) cell; negative when q
// lies outside the grid box, which only makes the stop bound more conservative
__device__ __forceinline__ double cell_margin(const GridView& g, float x, float y, float z, int cx, int cy,
                                              int cz) {
  double lx = (double)g.ox + (double)cx * g.h, ly = (double)g.oy + (double)cy * g.h,
         lz = (double)g.oz + (double)cz * g.h;
  double m = fmin(fmin((double)x - lx, lx + g.h - (double)x),
                  fmin(fmin((double)y - ly, ly + g.h - (double)y), fmin((double)z - lz, lz + g.h - (double)z)));
  return m;
}

// nanoflann L2_Adaptor::evalMetric (dim 3): ((dx*dx) + dy*dy) + dz*dz, double.
__device__ __forceinline__ double dist2_f64(double qx, double qy, double qz, float4 p) {
  double dx = qx - (double)p.x, dy = qy - (double)p.y, dz = qz - (double)p.z;
  double r = dx * dx;
  r = r + dy * dy;
  r = r + dz * dz;
  return r;
}

// Visit every cell of Chebyshev shell r around (cx,cy,cz); f(cell) per cell.
template <class F>
__device__ __forceinline__ void for_shell(const GridView& g, int cx, int cy, int cz, int r, F&& f) {
  for (int dz = -r; dz <= r; ++dz) {
    const int z = cz + dz;
    if (z < 0 || z >= g.nz) continue;
    const bool zf = (dz == -r) || (dz == r);
    for (int dy = -r; dy <= r; ++dy) {
      const int y = cy + dy;
      if (y < 0 || y >= g.ny) continue;
      const bool face = zf || (dy == -r) || (dy == r);
      const int step = face ? 1 : 2 * r;
      for (int dx = -r; dx <= r; dx += step) {
        const int x = cx + dx;
        if (x < 0 || x >= g.nx) continue;
        f(x + g.nx * (y + g.ny * z));
      }
    }
  }
}

__device__ __forceinline__ int shell_rmax(const GridView& g, int cx, int cy, int cz) {
  return max(max(max(cx, g.nx - 1 - cx), max(cy, g.ny - 1 - cy)), max(cz, g.nz - 1 - cz));
}

__device__ __forceinline__ bool lex_less(double d, int i, double bd, int bi) {
  return d < bd || (d == bd && i < bi);
}

// Sorted top-K (by (d2, sorted position)) neighbour search.  kneed <= K.
// mode: O3DX_SEARCH_KNN or O3DX_SEARCH_HYBRID (r2lim = radius^2, strict <).
// On return bd/bi[0..cnt) hold the neighbours, nearest first; bi are original
// point indices (ties in d^2 broken by the lower original index).
template <int K>
__device__ __forceinline__ int knn_search_dev(const GridView& g, float qx, float qy, float qz, int kneed,
                                              bool hybrid, double radius, double bd[K], int bi[K]) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    bd[j] = INFINITY;
    bi[j] = 0x7fffffff;
  }
  if (g.n == 0 || kneed <= 0) return 0;
  int cx, cy, cz;
  grid_cell(g, qx, qy, qz, cx, cy, cz);
  const double m = cell_margin(g, qx, qy, qz, cx, cy, cz);
  const int rmax = shell_rmax(g, cx, cy, cz);
  const double dqx = qx, dqy = qy, dqz = qz;
  const double r2lim = hybrid ? radius * radius : INFINITY;
  double wd = INFINITY;
  int wi = 0x7fffffff;
  int cnt = 0;
  for (int r = 0; r <= rmax; ++r) {
    for_shell(g, cx, cy, cz, r, [&](int c) {
      const int s1 = g.start[c + 1];
      for (int p = g.start[c]; p < s1; ++p) {
        const float4 v = g.pts[p];
        const double d = dist2_f64(dqx, dqy, dqz, v);
        if (!(d < r2lim)) continue;
        const int oi = __float_as_int(v.w);
        if (lex_less(d, oi, wd, wi)) {
#pragma unroll
          for (int j = K - 1; j >= 0; --j) {
            const bool lt = lex_less(d, oi, bd[j], bi[j]);
            const bool ltp = (j > 0) ? lex_less(d, oi, bd[j > 0 ? j - 1 : 0], bi[j > 0 ? j - 1 : 0]) : false;
            if (ltp) {
              bd[j] = bd[j - 1];
              bi[j] = bi[j - 1];
            } else if (lt) {
              bd[j] = d;
              bi[j] = oi;
            }
          }
          cnt = cnt < kneed ? cnt + 1 : kneed;
          if (cnt == kneed) {
#pragma unroll
            for (int j = 0; j < K; ++j)
              if (j == kneed - 1) {
                wd = bd[j];
                wi = bi[j];
              }
          }
        }
      }
    });
    const double B = (double)r * g.h + m - g.slack;
    if (cnt >= kneed && B > 0.0 && wd < B * B) break;
    if (hybrid && B >= radius) break;
  }
  return cnt;
}

// Nearest neighbour with d^2 < radius^2 (SearchHybrid(p, r, 1)); returns its
// original index, -1 if none.
__device__ __forceinline__ int nn_search_dev(const GridView& g, double qx, double qy, double qz, double radius,
                                             double* best_d2, int* best_pos) {
  double bd = INFINITY;
  int bi = -1, bp = -1;
  if (g.n == 0) {
    *best_d2 = bd;
    *best_pos = -1;
    return -1;
  }
  const float fx = (float)qx, fy = (float)qy, fz = (float)qz;
  int cx, cy, cz;
  // queries may lie outside the grid box: clamp, and account for the overshoot
  grid_cell(g, fx, fy, fz, cx, cy, cz);
  const double lx = (double)g.ox + (double)cx * g.h, ly = (double)g.oy + (double)cy * g.h,
               lz = (double)g.oz + (double)cz * g.h;
  double m = fmin(fmin(qx - lx, lx + g.h - qx), fmin(fmin(qy - ly, ly + g.h - qy), fmin(qz - lz, lz + g.h - qz)));
  // outside the query's cell (clamped): m < 0 shrinks the bound, still valid
  const int rmax = shell_rmax(g, cx, cy, cz);
  const double r2lim = radius * radius;
  for (int r = 0; r <= rmax; ++r) {
    for_shell(g, cx, cy, cz, r, [&](int c) {
      const int s1 = g.start[c + 1];
      for (int p = g.start[c]; p < s1; ++p) {
        const float4 v = g.pts[p];
        const double d = dist2_f64(qx, qy, qz, v);
        const int oi = __float_as_int(v.w);
        if (d < r2lim && lex_less(d, oi, bd, bi < 0 ? 0x7fffffff : bi)) {
          bd = d;
          bi = oi;
          bp = p;
        }
      }
    });
    const double B = (double)r * g.h + m - g.slack;
    if (B >= radius) break;
    if (bi >= 0 && B > 0.0 && bd < B * B) break;
  }
  *best_d2 = bd;
  *best_pos = bp;
  return bi;
}

// ---------------------------------------------------------------- build
struct GridBuild {
  // device buffers (carved from a workspace)
  float4* pts;
  float4* extra;  // per-point payload sorted like pts (ICP target normals), or null
  int32_t* start;
  int32_t* count;
  int32_t* cell;
  int32_t* rank;
  int32_t* scan_tmp;
  char* aabb_ws;
  double* mm;
  int64_t* scratch;
  int64_t cap_cells;
  GridView view;
};

size_t grid_ws_bytes(int64_t n);
// target_occ: desired mean points per occupied cell.  min_h: lower bound on h
// (0 = none).  Synchronises the stream (cell size is chosen on the host).
int grid_build(const float* xyz, int64_t n, double target_occ, double min_h, void* ws, size_t ws_bytes,
               hipStream_t s, GridBuild* out, float4* extra_sorted = nullptr, const float* extra_src = nullptr);

}  // namespace o3dx
