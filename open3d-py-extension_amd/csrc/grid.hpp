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

struct Mat4d {
  double m[16];
};

struct GridView {
  const float4* __restrict__ pts;      // sorted by cell: (x, y, z, bits(original index))
  const int32_t* __restrict__ start;   // ncells + 1
  float ox, oy, oz, h, inv_h;
  float slack;                         // conservative rounding margin for the stop test
  int nx, ny, nz;
  int64_t n;
  unsigned long long* stats;  // debug: {queries, cells visited, candidates, shells}; null = off
  int blocked;                // cell order: 0 = row-major (x fastest; searchable), 1 = 8^3 blocks
  int bnx, bny;               // blocked order: number of blocks along x, y
  int dense = 0;              // 1: pts is a dense voxel table (<= 1 point per cell, empty = NaN
                              // coordinates, w = -1) and start is the identity (start may be null)
  int32_t* nbr = nullptr;     // test hook (o3dx_set_debug_neighbors): k selected ids per output row
  float* kd2 = nullptr;       // KNN normals: per output row an upper bound of the k-th neighbour d^2
  // Nested grid (KNN normals on clouds of mixed density, grid.hip "nested
  // grids"): a finer grid over the dense cells of an outer grid and their
  // neighbours.  Its w = the point's outer sorted position when the point is a
  // query here, -(position + 1) when it is only a candidate.  Searches are
  // capped at the outer grid's shell-1 reach (every point inside it is here).
  const float4* __restrict__ outer = nullptr;
  float cox = 0.f, coy = 0.f, coz = 0.f, ch = 0.f, cinv_h = 0.f, cslack = 0.f;
  int cnx = 0, cny = 0, cnz = 0;
  const uint8_t* skip_cells = nullptr;  // outer grid: queries in flagged cells are the nested grid's
  // float64 clouds (f64.hip): pts holds float32(p - o64), the search frame
  // (cells, filters, reach tests; the float32 rounding of the frame is inside
  // `slack`); pts64 the exact float64 coordinates in the same sorted order, w
  // = the original index — every distance that decides is computed from them
  // in nanoflann's order, as Open3D computes it on its float64 storage.
  const double4* __restrict__ pts64 = nullptr;
  double o64x = 0.0, o64y = 0.0, o64z = 0.0;
  // |frame distance - exact distance| <= d64 (both points' float32 frame
  // roundings, 2 sqrt(3) half-ulps of the frame's largest magnitude)
  float d64 = 0.f;
  const double* __restrict__ xyz64 = nullptr;  // the caller's (n,3) float64 points (original order)
};

// outer sorted position / output row of a nested-grid point
__device__ __forceinline__ int nested_pos(int w) { return w >= 0 ? w : -w - 1; }
__device__ __forceinline__ int out_row(const GridView& g, int w) {
  return g.outer ? __float_as_int(g.outer[nested_pos(w)].w) : w;
}

// First sorted position of cell c (dense tables: the cell itself).
__device__ __forceinline__ int cell_start(const GridView& g, int c) { return g.dense ? c : g.start[c]; }

// Cell index.  Row-major (x fastest) keeps every (y,z) row contiguous, which
// the searches rely on.  The blocked order (spatial_sort only) lists 8x8x8
// blocks row-major and the cells of a block in Morton order, so consecutive
// points form compact 3-D patches on any surface.
__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 3 bits -> every third bit
  return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4);
}
__device__ __forceinline__ int cell_index(const GridView& g, int cx, int cy, int cz) {
  if (!g.blocked) return cx + g.nx * (cy + g.ny * cz);
  const int b = (cx >> 3) + g.bnx * ((cy >> 3) + g.bny * (cz >> 3));
  return (b << 9) | (int)(spread3(cx & 7) | (spread3(cy & 7) << 1) | (spread3(cz & 7) << 2));
}

__device__ __forceinline__ void search_stats(const GridView& g, int cells, int cands, int shells) {
  if (g.stats) {
    atomicAdd(&g.stats[0], 1ull);
    atomicAdd(&g.stats[1], (unsigned long long)cells);
    atomicAdd(&g.stats[2], (unsigned long long)cands);
    atomicAdd(&g.stats[3], (unsigned long long)shells);
  }
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ void grid_cell(const GridView& g, float x, float y, float z, int& cx, int& cy,
                                          int& cz) {
  cx = clampi((int)floorf((x - g.ox) * g.inv_h), 0, g.nx - 1);
  cy = clampi((int)floorf((y - g.oy) * g.inv_h), 0, g.ny - 1);
  cz = clampi((int)floorf((z - g.oz) * g.inv_h), 0, g.nz - 1);
}

// float32 squared distance (filtering only; decisions are made in float64)
__device__ __forceinline__ float dist2_f32(const float4 q, float x, float y, float z) {
  const float dx = q.x - x, dy = q.y - y, dz = q.z - z;
  return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
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

// Visit the cube of cells within Chebyshev distance S of (cx,cy,cz) as
// (2S+1)^2 row ranges: the cells of one (y,z) row are adjacent in the
// cell-sorted array, so each row of the cube is ONE contiguous point range
// [start[first], start[last+1]).  f(p0, p1) per row.
template <class F>
__device__ __forceinline__ void for_cube_rows(const GridView& g, int cx, int cy, int cz, int S, F&& f) {
  const int x0 = max(cx - S, 0), x1 = min(cx + S, g.nx - 1);
  for (int dz = -S; dz <= S; ++dz) {
    const int z = cz + dz;
    if (z < 0 || z >= g.nz) continue;
    for (int dy = -S; dy <= S; ++dy) {
      const int y = cy + dy;
      if (y < 0 || y >= g.ny) continue;
      const int rb = g.nx * (y + g.ny * z);
      f(cell_start(g, rb + x0), cell_start(g, rb + x1 + 1));
    }
  }
}

// f(p, point) over [p0, p1) with four loads in flight per step
template <class F>
__device__ __forceinline__ void for_points4(const GridView& g, int p0, int p1, F&& f) {
  int p = p0;
  for (; p + 4 <= p1; p += 4) {
    const float4 a = g.pts[p], b = g.pts[p + 1], c = g.pts[p + 2], d = g.pts[p + 3];
    f(p, a);
    f(p + 1, b);
    f(p + 2, c);
    f(p + 3, d);
  }
  for (; p < p1; ++p) f(p, g.pts[p]);
}

// Completeness radius of the (2S+1)^3 cube around cell (cx,cy,cz): the
// distance from q to the nearest cube face that has grid cells beyond it
// (faces on the grid boundary have no points beyond them: the grid covers
// every point, clamped).  Every point closer to q than this (minus the
// rounding slack) lies in the cube.  +inf when the cube covers the grid.
__device__ __forceinline__ double cube_reach(const GridView& g, double x, double y, double z, int cx, int cy, int cz,
                                             int S) {
  double r = INFINITY;
  if (cx - S > 0) r = fmin(r, x - ((double)g.ox + (double)(cx - S) * g.h));
  if (cx + S < g.nx - 1) r = fmin(r, ((double)g.ox + (double)(cx + S + 1) * g.h) - x);
  if (cy - S > 0) r = fmin(r, y - ((double)g.oy + (double)(cy - S) * g.h));
  if (cy + S < g.ny - 1) r = fmin(r, ((double)g.oy + (double)(cy + S + 1) * g.h) - y);
  if (cz - S > 0) r = fmin(r, z - ((double)g.oz + (double)(cz - S) * g.h));
  if (cz + S < g.nz - 1) r = fmin(r, ((double)g.oz + (double)(cz + S + 1) * g.h) - z);
  return r;
}

// A nested grid's cap: the outer grid's shell-1 completeness radius around q
// (minus the outer slack); +inf for an outer grid.
__device__ __forceinline__ double outer_reach(const GridView& g, double x, double y, double z) {
  if (!g.outer) return INFINITY;
  const int cx = clampi((int)floorf(((float)x - g.cox) * g.cinv_h), 0, g.cnx - 1);
  const int cy = clampi((int)floorf(((float)y - g.coy) * g.cinv_h), 0, g.cny - 1);
  const int cz = clampi((int)floorf(((float)z - g.coz) * g.cinv_h), 0, g.cnz - 1);
  double r = INFINITY;
  if (cx - 1 > 0) r = fmin(r, x - ((double)g.cox + (double)(cx - 1) * g.ch));
  if (cx + 1 < g.cnx - 1) r = fmin(r, ((double)g.cox + (double)(cx + 2) * g.ch) - x);
  if (cy - 1 > 0) r = fmin(r, y - ((double)g.coy + (double)(cy - 1) * g.ch));
  if (cy + 1 < g.cny - 1) r = fmin(r, ((double)g.coy + (double)(cy + 2) * g.ch) - y);
  if (cz - 1 > 0) r = fmin(r, z - ((double)g.coz + (double)(cz - 1) * g.ch));
  if (cz + 1 < g.cnz - 1) r = fmin(r, ((double)g.coz + (double)(cz + 2) * g.ch) - z);
  return r - (double)g.cslack;
}

__device__ __forceinline__ int shell_rmax(const GridView& g, int cx, int cy, int cz) {
  return max(max(max(cx, g.nx - 1 - cx), max(cy, g.ny - 1 - cy)), max(cz, g.nz - 1 - cz));
}

__device__ __forceinline__ bool lex_less(double d, int i, double bd, int bi) {
  return d < bd || (d == bd && i < bi);
}

// nanoflann's d^2 of a float64 grid point (GridView::pts64)
__device__ __forceinline__ double dist2_d4(double qx, double qy, double qz, const double4& p) {
  const double dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
  double r = dx * dx;
  r = r + dy * dy;
  r = r + dz * dz;
  return r;
}

// The deciding float64 d^2 of sorted point p (float32 grid point v): from the
// exact float64 coordinates on a float64 grid (q in the cloud's own frame),
// from v itself otherwise
template <bool F64>
__device__ __forceinline__ double exact_d2(const GridView& g, double qx, double qy, double qz, int p, const float4& v) {
  if constexpr (F64)
    return dist2_d4(qx, qy, qz, g.pts64[p]);
  else
    return dist2_f64(qx, qy, qz, v);
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
  const int rmax = shell_rmax(g, cx, cy, cz);
  const double dqx = qx, dqy = qy, dqz = qz;
  const double r2lim = hybrid ? radius * radius : INFINITY;
  double wd = INFINITY;
  int wi = 0x7fffffff;
  int cnt = 0;
  int st_cells = 0, st_cands = 0, r = 0;
  for (r = 0; r <= rmax; ++r) {
    for_shell(g, cx, cy, cz, r, [&](int c) {
      const int s1 = cell_start(g, c + 1);
      if (g.stats) {
        ++st_cells;
        st_cands += s1 - cell_start(g, c);
      }
      for (int p = cell_start(g, c); p < s1; ++p) {
        const float4 v = g.pts[p];
        const double d = dist2_f64(dqx, dqy, dqz, v);
        if (!(d < r2lim)) continue;  // NaN (an empty dense cell) fails too
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
    const double B = cube_reach(g, dqx, dqy, dqz, cx, cy, cz, r) - g.slack;
    if (cnt >= kneed && B > 0.0 && wd < B * B) break;
    if (hybrid && B >= radius) break;
  }
  search_stats(g, st_cells, st_cands, r + 1);
  return cnt;
}

// knn_search_dev on a float64 grid (GridView::pts64): q in the cloud's own
// frame, every candidate's d^2 from its exact float64 coordinates.  Paging:
// only candidates after (lo_d, lo_i) in (d^2, index) order are taken, so a
// radius search of any size is read off in sorted pages of K (the default
// (-1, -1) takes all).  Returns the count; bd/bi as knn_search_dev.
#ifndef O3DX_F64_BATCH
#define O3DX_F64_BATCH 2
#endif
template <int K>
__device__ __forceinline__ int knn_search_dev64(const GridView& g, double qx, double qy, double qz, int kneed,
                                                bool hybrid, double radius, double bd[K], int bi[K],
                                                double lo_d = -1.0, int lo_i = -1) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    bd[j] = INFINITY;
    bi[j] = 0x7fffffff;
  }
  if (g.n == 0 || kneed <= 0) return 0;
  const double gqx = qx - g.o64x, gqy = qy - g.o64y, gqz = qz - g.o64z;
  int cx, cy, cz;
  grid_cell(g, (float)gqx, (float)gqy, (float)gqz, cx, cy, cz);
  const int rmax = shell_rmax(g, cx, cy, cz);
  const double r2lim = hybrid ? radius * radius : INFINITY;
  double wd = INFINITY;
  int wi = 0x7fffffff;
  int cnt = 0;
  int st_cells = 0, st_cands = 0, r = 0;
  for (r = 0; r <= rmax; ++r) {
    for_shell(g, cx, cy, cz, r, [&](int c) {
      const int s1 = g.start[c + 1];
      if (g.stats) {
        ++st_cells;
        st_cands += s1 - g.start[c];
      }
      // O3DX_F64_BATCH candidates' loads in flight at once (the same visiting order)
      for (int p0 = g.start[c]; p0 < s1; p0 += O3DX_F64_BATCH) {
        double4 vv[O3DX_F64_BATCH];
#pragma unroll
        for (int u = 0; u < O3DX_F64_BATCH; ++u) vv[u] = g.pts64[min(p0 + u, s1 - 1)];
#pragma unroll
        for (int u = 0; u < O3DX_F64_BATCH; ++u) {
        if (p0 + u >= s1) break;
        const double4 v = vv[u];
        const double d = dist2_d4(qx, qy, qz, v);
        if (!(d < r2lim)) continue;
        const int oi = (int)v.w;
        if (!lex_less(lo_d, lo_i, d, oi)) continue;  // an earlier page's
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
      }
    });
    const double B = cube_reach(g, gqx, gqy, gqz, cx, cy, cz, r) - g.slack;
    if (cnt >= kneed && B > 0.0 && wd < B * B) break;
    if (hybrid && B >= radius) break;
  }
  search_stats(g, st_cells, st_cands, r + 1);
  return cnt;
}

// Nearest neighbour with d^2 < radius^2 (SearchHybrid(p, r, 1)); returns its
// original index, -1 if none.  Beyond the own cell the walk goes by (y, z)
// rows (below; round 2 measured it against a Chebyshev shell walk: every
// correspondence equal, 1094 -> 1150 ICP iterations/s; the shell walk was
// removed in round 5).
// SHARE: the lanes calling together share first bounds (below); every lane
// of the wave that runs the search must call it at once.
// F64: a float64 grid (GridView::pts64), q in the cloud's own frame.
// EXT (the ICP loop's skip proof, icp.hip k_icp_step): the search covers the
// ball of radius sqrt(best) + ext instead of sqrt(best), and *margin receives
// a lower bound of (distance of any other target point) - (best distance):
// every other point examined in that ball has its exact distance kept, every
// point not examined lies beyond it.  Same result (best) either way.
template <bool SHARE = false, bool F64 = false, bool EXT = false>
__device__ __forceinline__ int nn_search_dev(const GridView& g, double qx, double qy, double qz, double radius,
                                             double* best_d2, int* best_pos, int prior = -1, double ext = 0.0,
                                             double* margin = nullptr) {
  double bd = INFINITY;
  int bi = -1, bp = -1;
  double sd = INFINITY;  // EXT: smallest exact d^2 of the other examined points
  auto finish = [&]() {
    *best_d2 = bd;
    *best_pos = bp;
    if constexpr (EXT) {
      if (bi < 0) {
        *margin = 0.0;
      } else {
        const double db = sqrt(bd);
        *margin = fmin(sqrt(sd), db + ext) - db;
      }
    }
  };
  if (g.n == 0) {
    bp = -1;
    finish();
    return -1;
  }
  // q in the grid's frame (float64 grids: relative to o64)
  const double gqx = F64 ? qx - g.o64x : qx, gqy = F64 ? qy - g.o64y : qy, gqz = F64 ? qz - g.o64z : qz;
  const float fx = (float)gqx, fy = (float)gqy, fz = (float)gqz;
  int cx, cy, cz;
  // queries may lie outside the grid box: clamped to the nearest cell (cube_reach
  // only counts faces with cells beyond them, so the bound stays valid)
  grid_cell(g, fx, fy, fz, cx, cy, cz);
  const double r2lim = radius * radius;
  int st_cells = 0, st_cands = 0, r = 0;
  // Cells are visited shell by shell.  Everything is filtered in float32
  // against thr, a float32 bound that every point beating the current best
  // (or lying inside the radius while there is none) stays below: the float32
  // distance of a point is within delta = slack of its exact distance, so
  // thr = (sqrt(best) + 2 delta)^2.  Only candidates below thr are compared
  // in float64 — the exact lexicographic (d^2, index) minimum is kept.  A
  // cell is skipped when the float32 lower bound of its box (shrunk by 3
  // delta per axis) reaches thr.
  const float4 qf = make_float4(fx, fy, fz, 0.f);
  const double dl = 2.0 * (double)g.slack;
  auto bound_of = [&](double dist) { return (float)((dist + dl) * (dist + dl) * (1.0 + 1e-6)); };
  float thr = bound_of(radius);
  const float sl3 = 3.0f * g.slack;
  auto visit_point = [&](int p, const float4 v) {
    if (dist2_f32(qf, v.x, v.y, v.z) < thr) {
      const double d = exact_d2<F64>(g, qx, qy, qz, p, v);
      const int oi = __float_as_int(v.w);
      if (d < r2lim && lex_less(d, oi, bd, bi < 0 ? 0x7fffffff : bi)) {
        if (EXT) sd = fmin(sd, bd);  // the former best is another point now
        bd = d;
        bi = oi;
        bp = p;
        thr = bound_of(sqrt(d) + ext);
      } else if (EXT && oi != bi) {  // (the best itself may be visited twice)
        sd = fmin(sd, d);
      }
    }
  };
  auto visit_cell = [&](int x, int y, int z) {
    const float bx0 = g.ox + (float)x * g.h, by0 = g.oy + (float)y * g.h, bz0 = g.oz + (float)z * g.h;
    const float ex = fmaxf(fmaxf(bx0 - fx, fx - (bx0 + g.h)) - sl3, 0.0f);
    const float ey = fmaxf(fmaxf(by0 - fy, fy - (by0 + g.h)) - sl3, 0.0f);
    const float ez = fmaxf(fmaxf(bz0 - fz, fz - (bz0 + g.h)) - sl3, 0.0f);
    if (fmaf(ez, ez, fmaf(ey, ey, ex * ex)) >= thr) return;
    const int c = x + g.nx * (y + g.ny * z);
    const int p0 = g.start[c], p1 = g.start[c + 1];
    if (g.stats) {
      ++st_cells;
      st_cands += p1 - p0;
    }
    for_points4(g, p0, p1, visit_point);
  };
  // prior: a target position to start from (the previous ICP iteration's
  // match; any real point gives a valid bound, the result is the same)
  if (prior >= 0) visit_point(prior, g.pts[prior]);
  bool own_seen = false;
  if (bi < 0) {
    visit_cell(cx, cy, cz);
    own_seen = true;
  }
  if (SHARE) {
    // A lane without a match yet borrows the match of the nearest lane (by
    // lane index) that has one as its starting bound: the queries of a wave
    // are neighbours in a spatially sorted source, and any real target point
    // bounds the search (the result is the same) — it spares the clipped
    // ring walk that would only look for a first bound.  Ballot and shuffle
    // see the lanes calling here.
    const uint64_t have = __ballot(bi >= 0);
    const bool borrow = have && bi < 0;
    const int lane = (int)(threadIdx.x & 63);
    int src_lane = lane;
    if (borrow) {
      const uint64_t up = lane < 63 ? have >> (lane + 1) : 0ull, down = have & ((1ull << lane) - 1ull);
      const int du = up ? __ffsll((unsigned long long)up) : 64;         // distance to the next lane above
      const int dd = down ? lane - (63 - __clzll((long long)down)) : 64;  // ... below
      src_lane = du <= dd ? lane + du : lane - dd;
    }
    const int p = __shfl(bp, src_lane, 64);  // converged: the source lanes take part
    if (borrow && p >= 0) visit_point(p, g.pts[p]);
  }
  if (bi >= 0) {
    // A match in the own cell bounds the search: every better point lies in
    // the ball of radius sqrt(thr) (+ the assignment slack), so only the
    // cells that ball overlaps are visited (the bound only shrinks while they
    // are scanned), instead of the full shells around the cell.
    const float rb = sqrtf(thr) + sl3;
    const int x0 = max(0, (int)floorf((fx - rb - g.ox) * g.inv_h)), x1 = min(g.nx - 1, (int)floorf((fx + rb - g.ox) * g.inv_h));
    const int y0 = max(0, (int)floorf((fy - rb - g.oy) * g.inv_h)), y1 = min(g.ny - 1, (int)floorf((fy + rb - g.oy) * g.inv_h));
    const int z0 = max(0, (int)floorf((fz - rb - g.oz) * g.inv_h)), z1 = min(g.nz - 1, (int)floorf((fz + rb - g.oz) * g.inv_h));
    if ((x1 - x0) <= 2 && (y1 - y0) <= 2 && (z1 - z0) <= 2 && x0 <= cx && cx <= x1 && y0 <= cy && cy <= y1 &&
        z0 <= cz && cz <= z1) {
      for (int z = z0; z <= z1; ++z)
        for (int y = y0; y <= y1; ++y)
          for (int x = x0; x <= x1; ++x)
            if (!own_seen || x != cx || y != cy || z != cz) visit_cell(x, y, z);
      search_stats(g, st_cells, st_cands, 2);
      finish();
      return bi;
    }
  }
  {
    // Row-ring walk: the (y, z) rows of the cell grid in rings k = max(|y -
    // cy|, |z - cz|) = 0, 1, 2, ...; each row contributes the x-chord of the
    // bound ball (cells whose box, grown by the slack, comes closer than
    // sqrt(thr)) as ONE contiguous point range of the row-major cell array.
    // Ring k's rows all lie at least g_k from q across y or z, so once
    // (g_k - slack)^2 reaches thr no later row can hold a point below the
    // bound.  Per ring O(k) row tests instead of O(k^2) cell tests (the shell
    // walk below): the far-displaced queries of the first iterations.
    // Without a match yet the chord would span the whole radius, so a first
    // pass (CLIP) keeps each ring's chords inside its Chebyshev cube (x within
    // k of cx) and ends with the ring that finds a match: it only sets the
    // bound; the full pass after it alone decides (and is complete).
    const int kmax = max(max(cy, g.ny - 1 - cy), max(cz, g.nz - 1 - cz));
    const double inv_hd = 1.0 / (double)g.h;
    int rows = 0;
    auto ring_walk = [&](bool clip) {
      for (int k = 0; k <= kmax; ++k) {
        if (k > 0) {
          float gk = INFINITY;  // smallest y/z gap of ring k's rows to q (sides with rows only)
          if (cy - k >= 0) gk = fminf(gk, fy - (g.oy + (float)(cy - k + 1) * g.h));
          if (cy + k < g.ny) gk = fminf(gk, (g.oy + (float)(cy + k) * g.h) - fy);
          if (cz - k >= 0) gk = fminf(gk, fz - (g.oz + (float)(cz - k + 1) * g.h));
          if (cz + k < g.nz) gk = fminf(gk, (g.oz + (float)(cz + k) * g.h) - fz);
          const float e = gk - sl3;
          if (e > 0.0f && e * e >= thr) break;
        }
        for (int dz = -k; dz <= k; ++dz) {
          const int z = cz + dz;
          if (z < 0 || z >= g.nz) continue;
          const bool zedge = dz == -k || dz == k;
          const int step = (zedge || k == 0) ? 1 : 2 * k;
          for (int dy = -k; dy <= k; dy += step) {
            const int y = cy + dy;
            if (y < 0 || y >= g.ny) continue;
            const float by0 = g.oy + (float)y * g.h, bz0 = g.oz + (float)z * g.h;
            const float ey = fmaxf(fmaxf(by0 - fy, fy - (by0 + g.h)) - sl3, 0.0f);
            const float ez = fmaxf(fmaxf(bz0 - fz, fz - (bz0 + g.h)) - sl3, 0.0f);
            const float eyz = fmaf(ez, ez, ey * ey);
            if (eyz >= thr) continue;
            const double rx = (double)sqrtf(thr - eyz) + (double)sl3;
            int xa = max(0, (int)floor(((double)fx - rx - (double)g.ox) * inv_hd));
            int xb = min(g.nx - 1, (int)floor(((double)fx + rx - (double)g.ox) * inv_hd));
            if (clip && bi < 0) {
              xa = max(xa, cx - k);
              xb = min(xb, cx + k);
            }
            if (xa > xb) continue;
            const int rb = g.nx * (y + g.ny * z);
            const int p0 = g.start[rb + xa], p1 = g.start[rb + xb + 1];
            if (g.stats) {
              ++rows;
              st_cands += p1 - p0;
            }
            for_points4(g, p0, p1, visit_point);
          }
        }
        r = k;
        if (clip && bi >= 0) break;
      }
    };
    if (bi < 0) ring_walk(true);
    ring_walk(false);
    search_stats(g, st_cells + rows, st_cands, r + 1);
    finish();
    return bi;
  }
}

// ------------------------------------------------------------- LDS tiles
// A chunk = <= Q consecutive queries (spatially sorted).  Its neighbour region
// = bounding box of the queries' cells +-1, staged row by row into LDS: each
// (y,z) row of the box is one contiguous range of the cell-sorted array, so
// the staging loads are coalesced.  ccs[k*(nxr+1) + i] is the LDS offset of
// the first point of cell (x0+i) in box row k (i = nxr: end of the row).
struct TileBox {
  int x0, x1, y0, y1, z0, z1;
  int nxr;  // x1 - x0 + 1
  int nyr;  // y1 - y0 + 1
};

// Stage the box into LDS as three float arrays (x, y, z; the original index
// is not staged: the rare exact-tie test fetches it with tile_global_pos).
// Every thread of the block must call it.  Returns the number of staged
// points, or -1 if the box does not fit (PTS points / cs_cap cell-start slots
// / kMaxTileRows rows).  `rows` needs kMaxTileRows+1 ints, `rstart` kMaxTileRows.
// The row prefix is one wave scan; each thread issues all of its (at most
// PTS/BLOCK) global loads before the first LDS store.
constexpr int kMaxTileRows = 36;

// tp (nullable): also each slot's global sorted position (the float64 tiles
// fetch the exact coordinates of their members by it).
template <int BLOCK, int PTS>
__device__ __forceinline__ int stage_tile(const GridView& g, const TileBox& b, float* __restrict__ tx, float* __restrict__ ty,
                          float* __restrict__ tz, int32_t* __restrict__ ccs, int cs_cap, int32_t* __restrict__ rows,
                          int32_t* __restrict__ rstart, int32_t* __restrict__ tp = nullptr) {
  static_assert(BLOCK >= kMaxTileRows, "row scan needs one lane per row");
  const int nrows = b.nyr * (b.z1 - b.z0 + 1);
  const int w = b.nxr + 1;
  if (nrows > kMaxTileRows || nrows * w > cs_cap) return -1;  // uniform across the block
  for (int t = threadIdx.x; t < nrows * w; t += BLOCK) {
    const int k = t / w, i = t - k * w;
    const int y = b.y0 + k % b.nyr, z = b.z0 + k / b.nyr;
    ccs[t] = g.start[(b.x0 + i) + g.nx * (y + g.ny * z)];  // global position for now
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int k = threadIdx.x;
    const int r0 = k < nrows ? ccs[k * w] : 0;
    const int len = k < nrows ? ccs[k * w + b.nxr] - r0 : 0;
    const int inc = wave_incl_scan(len);
    if (k < nrows) {
      rows[k + 1] = inc;
      rstart[k] = r0;
    }
    if (k == 0) rows[0] = 0;
  }
  __syncthreads();
  const int total = rows[nrows];
  if (total > PTS) return -1;
  for (int t = threadIdx.x; t < nrows * w; t += BLOCK) {
    const int k = t / w;
    ccs[t] = rows[k] + (ccs[t] - rstart[k]);
  }
  constexpr int J = (PTS + BLOCK - 1) / BLOCK;
  float4 buf[J];
  int gp[J];
  int k = 0;  // f only grows, so the row index is carried along
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int f = threadIdx.x + j * BLOCK;
    if (f < total) {
      while (rows[k + 1] <= f) ++k;
      gp[j] = rstart[k] + (f - rows[k]);
      buf[j] = g.pts[gp[j]];
    }
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int f = threadIdx.x + j * BLOCK;
    if (f < total) {
      tx[f] = buf[j].x;
      ty[f] = buf[j].y;
      tz[f] = buf[j].z;
      if (tp) tp[f] = gp[j];
    }
  }
  __syncthreads();
  return total;
}

// Global (cell-sorted) position of LDS tile slot f.
__device__ __forceinline__ int tile_global_pos(const int32_t* rows, const int32_t* rstart, int f) {
  int k = 0;
  while (rows[k + 1] <= f) ++k;
  return rstart[k] + (f - rows[k]);
}

// Cube S=1 around (cx,cy,cz) inside a staged box: f(lds_p0, lds_p1) per row.
template <class F>
__device__ __forceinline__ void for_tile_rows(const TileBox& b, const int32_t* ccs, int cx, int cy, int cz, F&& f) {
  const int w = b.nxr + 1;
  const int xa = max(cx - 1, b.x0) - b.x0, xb = min(cx + 1, b.x1) - b.x0;
  for (int dz = -1; dz <= 1; ++dz) {
    const int z = cz + dz;
    if (z < b.z0 || z > b.z1) continue;
    for (int dy = -1; dy <= 1; ++dy) {
      const int y = cy + dy;
      if (y < b.y0 || y > b.y1) continue;
      const int k = (y - b.y0) + b.nyr * (z - b.z0);
      f(ccs[k * w + xa], ccs[k * w + xb + 1]);
    }
  }
}

// Chunk plan (normals tiles): the grid's own points in chunks of <= qcap
// consecutive queries: long (y,z) rows cut in qcap pieces, short rows of one z
// slab merged (within groups of 10 rows).  chunk_starts needs
// chunk_plan_upper()+2 entries; slots past the real count hold n.  Enqueues
// only (no host synchronisation).
int64_t chunk_plan_upper(int64_t n, const GridView& g, int qcap);
size_t chunk_plan_ws_bytes(int64_t n, int64_t rows);
int chunk_plan(int64_t n, const GridView& g, int qcap, int32_t* chunk_starts, void* ws, size_t ws_bytes,
               hipStream_t s);

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
  double4* pts64 = nullptr;  // float64 grids (grid64_build): exact coordinates + index, sorted like pts
  double mm_host[6] = {0, 0, 0, 0, 0, 0};  // the cloud's bounds (min xyz, max xyz), read back by grid_build
};

size_t grid_ws_bytes(int64_t n, int cap_mult = 4);
unsigned long long* search_stats_ptr();  // device counters when stats are enabled, else null
// target_occ: desired mean points per occupied cell.  min_h: lower bound on h
// (0 = none).  cap_mult: cell capacity per point (the workspace must come
// from grid_ws_bytes(n, cap_mult)).  Synchronises the stream (cell size is
// chosen on the host).
// ordered = false: points grouped by cell only (no ascending-index order
// inside a cell; for consumers that do not depend on it).
// ids: the w stored per point (default: its index; forces ordered = false).
// max_h: upper bound on h (0 = none).
// search.hip: stable radix sort of (cell key < 2^bits, point index) pairs
size_t cell_sort_temp_bytes(int64_t n, int bits);
int cell_sort(const uint32_t* key, uint32_t* skey, const int32_t* val, int32_t* sval, int64_t n, int bits, void* tmp,
              size_t tmp_bytes, hipStream_t s);
int grid_build(const float* xyz, int64_t n, double target_occ, double min_h, void* ws, size_t ws_bytes,
               hipStream_t s, GridBuild* out, float4* extra_sorted = nullptr, const float* extra_src = nullptr,
               bool blocked = false, int cap_mult = 4, bool ordered = true, const int32_t* ids = nullptr,
               double max_h = 0.0);

// Float64 clouds (include/o3dx.h "float64 boundary"): a grid over the
// float32 frame coordinates p - o (o = the cloud's float64 minimum bound),
// with the exact float64 coordinates sorted alongside (GridView::pts64, w =
// original index).  Workspace: grid64_ws_bytes.  extra_src: a float32 (n,3)
// payload sorted alongside (G.extra; ICP target normals).  mm_host
// (nullable): the cloud's {min, max} when the caller has it.
size_t grid64_ws_bytes(int64_t n, int cap_mult = 4);
int grid64_build(const double* xyz, int64_t n, double target_occ, double min_h, void* ws, size_t ws_bytes,
                 hipStream_t s, GridBuild* out, const float* extra_src = nullptr, int cap_mult = 4,
                 bool blocked = false, const double* mm_host = nullptr);

}  // namespace o3dx
