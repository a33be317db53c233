// oracle/o3d_restate.cpp — CPU restatement of the Open3D 0.19.0 algorithms the
// reference (qinhy/Open3D-py-extension) falls through to.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker /
// the CPU baseline — never as the product path.
//
// PARITY STATUS: "parity unpinned" for the Open3D-path functions in this file.
// The arithmetic lives in the third-party dependency open3d==0.19.0 (pinned at
// /root/reference/uv.lock:3108-3109, constraint pyproject.toml:10), which is
// absent from /root/reference and cannot be installed or built here, and the
// reference's own repository holds no golden vector, known-answer test or
// fixture for these calls (it has no asserting tests at all).
// The restatement follows Open3D's published algorithms; every [upstream]
// note names the Open3D source it restates.  The reference call sites each
// function serves are cited per function.
//
// Inputs are float64 coordinates, as Open3D stores them (Vector3dVector):
// a float32 cloud is passed upcast (exact), a float64 cloud as is (the
// float64 boundary of libo3dx, include/o3dx.h o3dx_*_f64).
//
// Floating-point order choices (documented so the GPU path can match them):
//   * voxel key  : ((double)p - min_bound) / voxel_size, floor, per axis.
//   * plane dist : (a*x + c*z) + (b*y + d)  — Eigen's packet reduction of a
//                  Vector4d dot (SSE2/AVX), no FMA.
//   * point d^2  : ((dx*dx) + dy*dy) + dz*dz in double (nanoflann L2_Adaptor).
//   * neighbour sets are ordered by (d^2, index) lexicographically; nanoflann
//     breaks exact distance ties by traversal order, which is unspecified.
//
// Build: oracle/Makefile (g++ -O3 -fopenmp -ffp-contract=off).

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <unordered_map>
#include <vector>
#include <omp.h>

namespace {

struct V3 {
  double x, y, z;
};

// ----------------------------------------------------------------- KD-tree
// Exact nearest-neighbour structure standing in for KDTreeFlann (nanoflann).
// Any exact kNN structure yields the same neighbour *set* (ties aside), which
// is all the covariance and ICP consume.
struct KDTree {
  struct Node {
    int lo, hi;       // range in perm
    int left, right;  // child nodes (-1 for leaf)
    double bmin[3], bmax[3];
  };
  const V3* pts = nullptr;
  std::vector<int> perm;
  std::vector<Node> nodes;
  static constexpr int kLeaf = 16;

  static double coord(const V3& p, int a) { return a == 0 ? p.x : (a == 1 ? p.y : p.z); }

  int build_rec(int lo, int hi) {
    Node nd;
    nd.lo = lo;
    nd.hi = hi;
    nd.left = nd.right = -1;
    for (int a = 0; a < 3; ++a) {
      nd.bmin[a] = std::numeric_limits<double>::infinity();
      nd.bmax[a] = -std::numeric_limits<double>::infinity();
    }
    for (int i = lo; i < hi; ++i) {
      const V3& p = pts[perm[i]];
      for (int a = 0; a < 3; ++a) {
        nd.bmin[a] = std::min(nd.bmin[a], coord(p, a));
        nd.bmax[a] = std::max(nd.bmax[a], coord(p, a));
      }
    }
    int id = (int)nodes.size();
    nodes.push_back(nd);
    if (hi - lo > kLeaf) {
      int axis = 0;
      double ext = nd.bmax[0] - nd.bmin[0];
      for (int a = 1; a < 3; ++a)
        if (nd.bmax[a] - nd.bmin[a] > ext) {
          ext = nd.bmax[a] - nd.bmin[a];
          axis = a;
        }
      int mid = (lo + hi) / 2;
      std::nth_element(perm.begin() + lo, perm.begin() + mid, perm.begin() + hi,
                       [&](int u, int v) { return coord(pts[u], axis) < coord(pts[v], axis); });
      int l = build_rec(lo, mid);
      int r = build_rec(mid, hi);
      nodes[id].left = l;
      nodes[id].right = r;
    }
    return id;
  }

  void build(const V3* p, int n) {
    pts = p;
    perm.resize(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    nodes.clear();
    nodes.reserve(2 * (n / kLeaf + 1) + 8);
    if (n > 0) build_rec(0, n);
  }

  static double box_d2(const Node& nd, const V3& q) {
    double s = 0.0;
    double qa[3] = {q.x, q.y, q.z};
    for (int a = 0; a < 3; ++a) {
      double d = 0.0;
      if (qa[a] < nd.bmin[a]) d = nd.bmin[a] - qa[a];
      else if (qa[a] > nd.bmax[a]) d = qa[a] - nd.bmax[a];
      s += d * d;
    }
    return s;
  }

  // nanoflann L2_Adaptor::evalMetric for dim 3: ((0 + dx^2) + dy^2) + dz^2
  static double dist2(const V3& q, const V3& p) {
    double dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
    double r = dx * dx;
    r = r + dy * dy;
    r = r + dz * dz;
    return r;
  }

  // Bounded sorted result set, lexicographic (d2, idx).
  struct KSet {
    int cap, cnt = 0;
    std::vector<double> d;
    std::vector<int> id;
    explicit KSet(int k) : cap(k), d(k, std::numeric_limits<double>::infinity()), id(k, -1) {}
    bool less(double d2, int i, int slot) const {
      return d2 < d[slot] || (d2 == d[slot] && i < id[slot]);
    }
    double worst() const { return cnt < cap ? std::numeric_limits<double>::infinity() : d[cap - 1]; }
    void add(double d2, int i) {
      if (cnt == cap && !less(d2, i, cap - 1)) return;
      int pos = cnt < cap ? cnt : cap - 1;
      while (pos > 0 && less(d2, i, pos - 1)) {
        d[pos] = d[pos - 1];
        id[pos] = id[pos - 1];
        --pos;
      }
      d[pos] = d2;
      id[pos] = i;
      if (cnt < cap) ++cnt;
    }
  };

  void knn_rec(int node, const V3& q, KSet& rs) const {
    const Node& nd = nodes[node];
    if (nd.left < 0) {
      for (int i = nd.lo; i < nd.hi; ++i) {
        int pi = perm[i];
        rs.add(dist2(q, pts[pi]), pi);
      }
      return;
    }
    const Node& L = nodes[nd.left];
    const Node& R = nodes[nd.right];
    double dl = box_d2(L, q), dr = box_d2(R, q);
    if (dl <= dr) {
      if (dl <= rs.worst()) knn_rec(nd.left, q, rs);
      if (dr <= rs.worst()) knn_rec(nd.right, q, rs);
    } else {
      if (dr <= rs.worst()) knn_rec(nd.right, q, rs);
      if (dl <= rs.worst()) knn_rec(nd.left, q, rs);
    }
  }

  void radius_rec(int node, const V3& q, double r2, std::vector<std::pair<double, int>>& out) const {
    const Node& nd = nodes[node];
    if (box_d2(nd, q) >= r2) return;
    if (nd.left < 0) {
      for (int i = nd.lo; i < nd.hi; ++i) {
        int pi = perm[i];
        double d2 = dist2(q, pts[pi]);
        if (d2 < r2) out.emplace_back(d2, pi);  // nanoflann RadiusResultSet: dist < radius
      }
      return;
    }
    radius_rec(nd.left, q, r2, out);
    radius_rec(nd.right, q, r2, out);
  }

  // KDTreeFlann::Search dispatch.  mode 0 KNN, 1 RADIUS, 2 HYBRID.
  // [upstream] KDTreeFlann.cpp SearchKNN / SearchRadius (sorted) /
  // SearchHybrid (= knnSearch(max_nn) truncated at lower_bound(r^2)).
  int search(const V3& q, int mode, int knn, double radius, std::vector<int>& idx,
             std::vector<double>& d2) const {
    idx.clear();
    d2.clear();
    if (nodes.empty()) return 0;
    if (mode == 1) {
      std::vector<std::pair<double, int>> out;
      radius_rec(0, q, radius * radius, out);
      std::sort(out.begin(), out.end());
      for (auto& e : out) {
        d2.push_back(e.first);
        idx.push_back(e.second);
      }
      return (int)idx.size();
    }
    int k = knn;
    if (k <= 0) return 0;
    KSet rs(k);
    knn_rec(0, q, rs);
    double r2 = radius * radius;
    for (int i = 0; i < rs.cnt; ++i) {
      if (mode == 2 && !(rs.d[i] < r2)) break;
      d2.push_back(rs.d[i]);
      idx.push_back(rs.id[i]);
    }
    return (int)idx.size();
  }
};

std::vector<V3> to_v3(const double* xyz, int64_t n) {
  std::vector<V3> v((size_t)n);
  for (int64_t i = 0; i < n; ++i) v[i] = {(double)xyz[3 * i], (double)xyz[3 * i + 1], (double)xyz[3 * i + 2]};
  return v;
}

// ----------------------------------------------------------- eigen helpers
// [upstream] utility/Eigen.cpp ComputeCovariance (raw moments, 9 cumulants).
void compute_covariance(const V3* pts, const int* idx, int k, double c[6] /*xx xy xz yy yz zz*/) {
  if (k == 0) {
    c[0] = 1; c[1] = 0; c[2] = 0; c[3] = 1; c[4] = 0; c[5] = 0;
    return;
  }
  double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const V3& p = pts[idx[j]];
    m[0] += p.x;
    m[1] += p.y;
    m[2] += p.z;
    m[3] += p.x * p.x;
    m[4] += p.x * p.y;
    m[5] += p.x * p.z;
    m[6] += p.y * p.y;
    m[7] += p.y * p.z;
    m[8] += p.z * p.z;
  }
  for (int j = 0; j < 9; ++j) m[j] /= (double)k;
  c[0] = m[3] - m[0] * m[0];
  c[3] = m[6] - m[1] * m[1];
  c[5] = m[8] - m[2] * m[2];
  c[1] = m[4] - m[0] * m[1];
  c[2] = m[5] - m[0] * m[2];
  c[4] = m[7] - m[1] * m[2];
}

struct M3 {
  double a[3][3];
};

void cross(const double u[3], const double v[3], double o[3]) {
  o[0] = u[1] * v[2] - u[2] * v[1];
  o[1] = u[2] * v[0] - u[0] * v[2];
  o[2] = u[0] * v[1] - u[1] * v[0];
}
double dot3(const double u[3], const double v[3]) { return (u[0] * v[0] + u[1] * v[1]) + u[2] * v[2]; }

// [upstream] geometry/EstimateNormals.cpp ComputeEigenvector0
void eigvec0(const M3& A, double eval0, double out[3]) {
  double r0[3] = {A.a[0][0] - eval0, A.a[0][1], A.a[0][2]};
  double r1[3] = {A.a[0][1], A.a[1][1] - eval0, A.a[1][2]};
  double r2[3] = {A.a[0][2], A.a[1][2], A.a[2][2] - eval0};
  double r0xr1[3], r0xr2[3], r1xr2[3];
  cross(r0, r1, r0xr1);
  cross(r0, r2, r0xr2);
  cross(r1, r2, r1xr2);
  double d0 = dot3(r0xr1, r0xr1), d1 = dot3(r0xr2, r0xr2), d2 = dot3(r1xr2, r1xr2);
  double dmax = d0;
  int imax = 0;
  if (d1 > dmax) {
    dmax = d1;
    imax = 1;
  }
  if (d2 > dmax) imax = 2;
  const double* v = imax == 0 ? r0xr1 : (imax == 1 ? r0xr2 : r1xr2);
  double s = std::sqrt(imax == 0 ? d0 : (imax == 1 ? d1 : d2));
  out[0] = v[0] / s;
  out[1] = v[1] / s;
  out[2] = v[2] / s;
}

// [upstream] geometry/EstimateNormals.cpp ComputeEigenvector1
void eigvec1(const M3& A, const double e0[3], double eval1, double out[3]) {
  double U[3], V[3];
  if (std::fabs(e0[0]) > std::fabs(e0[1])) {
    double inv = 1.0 / std::sqrt(e0[0] * e0[0] + e0[2] * e0[2]);
    U[0] = -e0[2] * inv;
    U[1] = 0;
    U[2] = e0[0] * inv;
  } else {
    double inv = 1.0 / std::sqrt(e0[1] * e0[1] + e0[2] * e0[2]);
    U[0] = 0;
    U[1] = e0[2] * inv;
    U[2] = -e0[1] * inv;
  }
  cross(e0, U, V);
  double AU[3] = {A.a[0][0] * U[0] + A.a[0][1] * U[1] + A.a[0][2] * U[2],
                  A.a[0][1] * U[0] + A.a[1][1] * U[1] + A.a[1][2] * U[2],
                  A.a[0][2] * U[0] + A.a[1][2] * U[1] + A.a[2][2] * U[2]};
  double AV[3] = {A.a[0][0] * V[0] + A.a[0][1] * V[1] + A.a[0][2] * V[2],
                  A.a[0][1] * V[0] + A.a[1][1] * V[1] + A.a[1][2] * V[2],
                  A.a[0][2] * V[0] + A.a[1][2] * V[1] + A.a[2][2] * V[2]};
  double m00 = U[0] * AU[0] + U[1] * AU[1] + U[2] * AU[2] - eval1;
  double m01 = U[0] * AV[0] + U[1] * AV[1] + U[2] * AV[2];
  double m11 = V[0] * AV[0] + V[1] * AV[1] + V[2] * AV[2] - eval1;
  double a00 = std::fabs(m00), a01 = std::fabs(m01), a11 = std::fabs(m11);
  if (a00 >= a11) {
    double mx = std::max(a00, a01);
    if (mx > 0) {
      if (a00 >= a01) {
        m01 /= m00;
        m00 = 1 / std::sqrt(1 + m01 * m01);
        m01 *= m00;
      } else {
        m00 /= m01;
        m01 = 1 / std::sqrt(1 + m00 * m00);
        m00 *= m01;
      }
      for (int i = 0; i < 3; ++i) out[i] = m01 * U[i] - m00 * V[i];
    } else {
      for (int i = 0; i < 3; ++i) out[i] = U[i];
    }
  } else {
    double mx = std::max(a11, a01);
    if (mx > 0) {
      if (a11 >= a01) {
        m01 /= m11;
        m11 = 1 / std::sqrt(1 + m01 * m01);
        m01 *= m11;
      } else {
        m11 /= m01;
        m01 = 1 / std::sqrt(1 + m11 * m11);
        m11 *= m01;
      }
      for (int i = 0; i < 3; ++i) out[i] = m11 * U[i] - m01 * V[i];
    } else {
      for (int i = 0; i < 3; ++i) out[i] = U[i];
    }
  }
}

// [upstream] geometry/EstimateNormals.cpp FastEigen3x3 (Eberly, robust 3x3
// symmetric eigensolver) -> eigenvector of the smallest eigenvalue.
// `nudge` (test certificates only; 0 = Open3D exactly): base-3 digits for the
// acos, cos(angle) and cos(angle + 2pi/3) results — 0 as is, 1 one ulp up,
// 2 one ulp down — the 1-ulp libm latitude between two correct platforms.
static double nudged(double v, int d) {
  return d == 1 ? std::nextafter(v, INFINITY) : d == 2 ? std::nextafter(v, -INFINITY) : v;
}

void fast_eigen3x3(const double c[6], double out[3], int nudge = 0) {
  M3 A;
  A.a[0][0] = c[0]; A.a[0][1] = c[1]; A.a[0][2] = c[2];
  A.a[1][0] = c[1]; A.a[1][1] = c[3]; A.a[1][2] = c[4];
  A.a[2][0] = c[2]; A.a[2][1] = c[4]; A.a[2][2] = c[5];
  double max_coeff = A.a[0][0];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) max_coeff = std::max(max_coeff, A.a[i][j]);
  if (max_coeff == 0) {
    out[0] = out[1] = out[2] = 0;
    return;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A.a[i][j] /= max_coeff;
  double norm = A.a[0][1] * A.a[0][1] + A.a[0][2] * A.a[0][2] + A.a[1][2] * A.a[1][2];
  if (norm > 0) {
    double q = (A.a[0][0] + A.a[1][1] + A.a[2][2]) / 3;
    double b00 = A.a[0][0] - q, b11 = A.a[1][1] - q, b22 = A.a[2][2] - q;
    double p = std::sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2) / 6);
    double c00 = b11 * b22 - A.a[1][2] * A.a[1][2];
    double c01 = A.a[0][1] * b22 - A.a[1][2] * A.a[0][2];
    double c02 = A.a[0][1] * A.a[1][2] - b11 * A.a[0][2];
    double det = (b00 * c00 - A.a[0][1] * c01 + A.a[0][2] * c02) / (p * p * p);
    double half_det = det * 0.5;
    half_det = std::min(std::max(half_det, -1.0), 1.0);
    double angle = nudged(std::acos(half_det), nudge % 3) / (double)3;
    const double two_thirds_pi = 2.09439510239319549;
    double beta2 = nudged(std::cos(angle), (nudge / 3) % 3) * 2;
    double beta0 = nudged(std::cos(angle + two_thirds_pi), (nudge / 9) % 3) * 2;
    double beta1 = -(beta0 + beta2);
    double eval[3] = {q + p * beta0, q + p * beta1, q + p * beta2};
    double e0[3], e1[3], e2[3];
    if (half_det >= 0) {
      eigvec0(A, eval[2], e2);
      if (eval[2] < eval[0] && eval[2] < eval[1]) {
        std::memcpy(out, e2, sizeof(e2));
        return;
      }
      eigvec1(A, e2, eval[1], e1);
      if (eval[1] < eval[0] && eval[1] < eval[2]) {
        std::memcpy(out, e1, sizeof(e1));
        return;
      }
      cross(e1, e2, out);
      return;
    } else {
      eigvec0(A, eval[0], e0);
      if (eval[0] < eval[1] && eval[0] < eval[2]) {
        std::memcpy(out, e0, sizeof(e0));
        return;
      }
      eigvec1(A, e0, eval[1], e1);
      if (eval[1] < eval[0] && eval[1] < eval[2]) {
        std::memcpy(out, e1, sizeof(e1));
        return;
      }
      cross(e0, e1, out);
      return;
    }
  } else {
    if (A.a[0][0] < A.a[1][1] && A.a[0][0] < A.a[2][2]) {
      out[0] = 1; out[1] = 0; out[2] = 0;
    } else if (A.a[1][1] < A.a[0][0] && A.a[1][1] < A.a[2][2]) {
      out[0] = 0; out[1] = 1; out[2] = 0;
    } else {
      out[0] = 0; out[1] = 0; out[2] = 1;
    }
  }
}

// Eigen Vector4d dot, packet order: (a*x + c*z) + (b*y + d*1)
inline double plane_dist_signed(const double pl[4], const V3& p) {
  double ax = pl[0] * p.x, by = pl[1] * p.y, cz = pl[2] * p.z, dw = pl[3] * 1.0;
  return (ax + cz) + (by + dw);
}

// [upstream] geometry/TriangleMesh.cpp ComputeTrianglePlane
void triangle_plane(const V3& p0, const V3& p1, const V3& p2, double pl[4]) {
  double e0[3] = {p1.x - p0.x, p1.y - p0.y, p1.z - p0.z};
  double e1[3] = {p2.x - p0.x, p2.y - p0.y, p2.z - p0.z};
  double abc[3];
  cross(e0, e1, abc);
  double norm = std::sqrt(dot3(abc, abc));
  if (norm == 0) {
    pl[0] = pl[1] = pl[2] = pl[3] = 0;
    return;
  }
  for (int i = 0; i < 3; ++i) abc[i] /= norm;
  double p0a[3] = {p0.x, p0.y, p0.z};
  double d = -dot3(abc, p0a);
  pl[0] = abc[0];
  pl[1] = abc[1];
  pl[2] = abc[2];
  pl[3] = d;
}

// [upstream] geometry/PointCloudSegmentation.cpp GetPlaneFromPoints, from the
// centroid and centred second moments.
void plane_from_moments(const double centroid[3], double xx, double xy, double xz, double yy,
                        double yz, double zz, double pl[4]) {
  double det_x = yy * zz - yz * yz;
  double det_y = xx * zz - xz * xz;
  double det_z = xx * yy - xy * xy;
  double abc[3];
  if (det_x > det_y && det_x > det_z) {
    abc[0] = det_x; abc[1] = xz * yz - xy * zz; abc[2] = xy * yz - xz * yy;
  } else if (det_y > det_z) {
    abc[0] = xz * yz - xy * zz; abc[1] = det_y; abc[2] = xy * xz - yz * xx;
  } else {
    abc[0] = xy * yz - xz * yy; abc[1] = xy * xz - yz * xx; abc[2] = det_z;
  }
  double norm = std::sqrt(dot3(abc, abc));
  if (norm == 0) {
    pl[0] = pl[1] = pl[2] = pl[3] = 0;
    return;
  }
  for (int i = 0; i < 3; ++i) abc[i] /= norm;
  pl[0] = abc[0];
  pl[1] = abc[1];
  pl[2] = abc[2];
  pl[3] = -dot3(abc, centroid);
}

void plane_from_points(const V3* pts, const int64_t* idx, int64_t k, double pl[4]) {
  double c[3] = {0, 0, 0};
  for (int64_t j = 0; j < k; ++j) {
    const V3& p = pts[idx[j]];
    c[0] += p.x;
    c[1] += p.y;
    c[2] += p.z;
  }
  for (int i = 0; i < 3; ++i) c[i] /= (double)k;
  double xx = 0, xy = 0, xz = 0, yy = 0, yz = 0, zz = 0;
  for (int64_t j = 0; j < k; ++j) {
    const V3& p = pts[idx[j]];
    double r0 = p.x - c[0], r1 = p.y - c[1], r2 = p.z - c[2];
    xx += r0 * r0;
    xy += r0 * r1;
    xz += r0 * r2;
    yy += r1 * r1;
    yz += r1 * r2;
    zz += r2 * r2;
  }
  plane_from_moments(c, xx, xy, xz, yy, yz, zz, pl);
}

// Eigen-style LDLT with diagonal pivoting for the 6x6 ICP system; zero pivots
// give zero solution components (Eigen LDLT::solve).
bool ldlt_solve6(const double A_in[36], const double b_in[6], double x[6]) {
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
    double dk = A[k * n + k];
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

// [upstream] utility/Eigen.cpp TransformVector6dToMatrix4d:
// R = AngleAxis(x2,Z) * AngleAxis(x1,Y) * AngleAxis(x0,X), t = x[3..5].
void vec6_to_mat4(const double x[6], double T[16]) {
  double ca = std::cos(x[0]), sa = std::sin(x[0]);
  double cb = std::cos(x[1]), sb = std::sin(x[1]);
  double cg = std::cos(x[2]), sg = std::sin(x[2]);
  double Rz[9] = {cg, -sg, 0, sg, cg, 0, 0, 0, 1};
  double Ry[9] = {cb, 0, sb, 0, 1, 0, -sb, 0, cb};
  double Rx[9] = {1, 0, 0, 0, ca, -sa, 0, sa, ca};
  double RzRy[9], R[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      RzRy[i * 3 + j] = (Rz[i * 3 + 0] * Ry[0 * 3 + j] + Rz[i * 3 + 1] * Ry[1 * 3 + j]) + Rz[i * 3 + 2] * Ry[2 * 3 + j];
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      R[i * 3 + j] = (RzRy[i * 3 + 0] * Rx[0 * 3 + j] + RzRy[i * 3 + 1] * Rx[1 * 3 + j]) + RzRy[i * 3 + 2] * Rx[2 * 3 + j];
    }
  for (int i = 0; i < 16; ++i) T[i] = 0;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) T[i * 4 + j] = R[i * 3 + j];
    T[i * 4 + 3] = x[3 + i];
  }
  T[15] = 1;
}

void mat4_mul(const double A[16], const double B[16], double C[16]) {
  double t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      t[i * 4 + j] = ((A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j]) + A[i * 4 + 2] * B[2 * 4 + j]) +
                     A[i * 4 + 3] * B[3 * 4 + j];
  std::memcpy(C, t, sizeof(t));
}

void transform_points(const double T[16], std::vector<V3>& pts) {
  for (auto& p : pts) {
    double x = p.x, y = p.y, z = p.z;
    double nx = ((T[0] * x + T[1] * y) + T[2] * z) + T[3];
    double ny = ((T[4] * x + T[5] * y) + T[6] * z) + T[7];
    double nz = ((T[8] * x + T[9] * y) + T[10] * z) + T[11];
    double nw = ((T[12] * x + T[13] * y) + T[14] * z) + T[15];
    p = {nx / nw, ny / nw, nz / nw};
  }
}

}  // namespace

extern "C" {

int oref_num_threads(void) { return omp_get_max_threads(); }
void oref_set_num_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

// Reference: PointCloud.get_aabb (PointCloud.py:145-146).  [upstream]
// Geometry3D::ComputeMinBound/MaxBound (zero vector for an empty cloud).
void oref_aabb(const double* xyz, int64_t n, double* mm) {
  if (n == 0) {
    for (int i = 0; i < 6; ++i) mm[i] = 0;
    return;
  }
  for (int a = 0; a < 3; ++a) {
    mm[a] = xyz[a];
    mm[3 + a] = xyz[a];
  }
  for (int64_t i = 1; i < n; ++i)
    for (int a = 0; a < 3; ++a) {
      double v = xyz[3 * i + a];
      mm[a] = std::min(mm[a], v);
      mm[3 + a] = std::max(mm[3 + a], v);
    }
}

// Reference: voxel_down_sample_and_trace (PointCloud.py:338-341) +
// idxmat.max(1) + _select_by_idx (:185-204).  [upstream]
// PointCloud::VoxelDownSampleAndTrace: single pass over points in index order,
// unordered_map<Vector3i, AccumulatedPointForTrace>; cubic id bit c set when
// (ref_coord - floor) >= 0.5; cubic_id(row, cid) = last (= max) index seen in
// that octant.  Output rows here are ordered by ascending representative
// (= max) index, the order _select_by_idx produces.
// Returns 0, or -22 on Open3D's LogError conditions.
int oref_voxel_down_sample(const double* xyz, int64_t n, const double* minb, const double* maxb,
                           double vs, int32_t* rep_idx, int64_t* m_out, int32_t* voxel_of_point,
                           int32_t* cubic) {
  if (vs <= 0.0) return -22;
  double ext = std::max(maxb[0] - minb[0], std::max(maxb[1] - minb[1], maxb[2] - minb[2]));
  if (vs * (double)std::numeric_limits<int>::max() < ext) return -22;
  struct Key {
    int x, y, z;
    bool operator==(const Key& o) const { return x == o.x && y == o.y && z == o.z; }
  };
  struct KH {
    size_t operator()(const Key& k) const {
      // [upstream] utility::hash_eigen: boost-style hash_combine
      size_t seed = 0;
      for (int v : {k.x, k.y, k.z}) seed ^= std::hash<int>()(v) + 0x9e3779b9 + (seed << 6) + (seed >> 2);
      return seed;
    }
  };
  struct Acc {
    int32_t last[8];
    int32_t maxi;
    int32_t row;
  };
  std::unordered_map<Key, int32_t, KH> map;  // key -> slot in accs
  std::vector<Acc> accs;
  std::vector<int32_t> slot_of((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    double ref[3];
    int vi[3];
    for (int a = 0; a < 3; ++a) {
      ref[a] = ((double)xyz[3 * i + a] - minb[a]) / vs;
      vi[a] = (int)std::floor(ref[a]);
    }
    int cid = 0;
    const int cid_temp[3] = {1, 2, 4};
    for (int a = 0; a < 3; ++a)
      if ((ref[a] - vi[a]) >= 0.5) cid += cid_temp[a];
    Key k{vi[0], vi[1], vi[2]};
    auto it = map.find(k);
    int32_t s;
    if (it == map.end()) {
      s = (int32_t)accs.size();
      map.emplace(k, s);
      Acc a;
      for (int c = 0; c < 8; ++c) a.last[c] = -1;
      a.maxi = -1;
      a.row = -1;
      accs.push_back(a);
    } else {
      s = it->second;
    }
    accs[s].last[cid] = (int32_t)i;
    accs[s].maxi = (int32_t)i;
    slot_of[i] = s;
  }
  std::vector<int32_t> reps;
  reps.reserve(accs.size());
  for (auto& a : accs) reps.push_back(a.maxi);
  std::sort(reps.begin(), reps.end());
  // row of each slot
  for (size_t r = 0; r < reps.size(); ++r) accs[slot_of[reps[r]]].row = (int32_t)r;
  for (size_t r = 0; r < reps.size(); ++r) rep_idx[r] = reps[r];
  *m_out = (int64_t)reps.size();
  if (voxel_of_point)
    for (int64_t i = 0; i < n; ++i) voxel_of_point[i] = accs[slot_of[i]].row;
  if (cubic)
    for (auto& a : accs)
      for (int c = 0; c < 8; ++c) cubic[(size_t)a.row * 8 + c] = a.last[c];
  return 0;
}

// The representatives of oref_voxel_down_sample (max index per voxel key,
// ascending) computed in parallel for clouds too large for the single pass
// (200M points: minutes).  Same key formula; points are split into buckets by
// a hash of their key (per-thread chunks keep each bucket's indices
// ascending), each bucket keeps the last = max index per key.  The function
// of the input is the same as the single pass's rep_idx; the CPU suite holds
// the two equal.
int oref_voxel_reps_parallel(const double* xyz, int64_t n, const double* minb, const double* maxb, double vs,
                             int32_t* rep_idx, int64_t* m_out) {
  if (vs <= 0.0) return -22;
  double ext = std::max(maxb[0] - minb[0], std::max(maxb[1] - minb[1], maxb[2] - minb[2]));
  if (vs * (double)std::numeric_limits<int>::max() < ext) return -22;
  constexpr int kB = 4096;
  auto key_of = [&](int64_t i, int64_t* k3) {
    for (int a = 0; a < 3; ++a) k3[a] = (int64_t)std::floor(((double)xyz[3 * i + a] - minb[a]) / vs);
  };
  auto bucket_of = [](const int64_t* k3) {
    uint64_t h = (uint64_t)k3[0] * 0x9E3779B97F4A7C15ull ^ (uint64_t)k3[1] * 0xC2B2AE3D27D4EB4Full ^
                 (uint64_t)k3[2] * 0x165667B19E3779F9ull;
    h ^= h >> 29;
    return (int)(h % kB);
  };
  const int T = omp_get_max_threads();
  std::vector<uint16_t> bk((size_t)n);
  std::vector<int64_t> cnt((size_t)T * kB, 0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const int64_t a = n * t / T, b = n * (t + 1) / T;
    int64_t* c = &cnt[(size_t)t * kB];
    for (int64_t i = a; i < b; ++i) {
      int64_t k3[3];
      key_of(i, k3);
      const int h = bucket_of(k3);
      bk[i] = (uint16_t)h;
      ++c[h];
    }
  }
  // offsets: bucket-major, thread-minor (so a bucket's indices stay ascending)
  std::vector<int64_t> start((size_t)kB + 1, 0);
  int64_t run = 0;
  for (int h = 0; h < kB; ++h) {
    start[h] = run;
    for (int t = 0; t < T; ++t) {
      const int64_t v = cnt[(size_t)t * kB + h];
      cnt[(size_t)t * kB + h] = run;
      run += v;
    }
  }
  start[kB] = run;
  std::vector<int32_t> order((size_t)n);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const int64_t a = n * t / T, b = n * (t + 1) / T;
    int64_t* c = &cnt[(size_t)t * kB];
    for (int64_t i = a; i < b; ++i) order[c[bk[i]]++] = (int32_t)i;
  }
  std::vector<std::vector<int32_t>> out(kB);
#pragma omp parallel for schedule(dynamic, 8) num_threads(T)
  for (int h = 0; h < kB; ++h) {
    struct K3 {
      int64_t x, y, z;
      bool operator==(const K3& o) const { return x == o.x && y == o.y && z == o.z; }
    };
    struct KH3 {
      size_t operator()(const K3& k) const {
        return (size_t)(k.x * 73856093 ^ k.y * 19349663 ^ k.z * 83492791);
      }
    };
    std::unordered_map<K3, int32_t, KH3> last;
    last.reserve((size_t)(start[h + 1] - start[h]));
    for (int64_t j = start[h]; j < start[h + 1]; ++j) {
      int64_t k3[3];
      key_of(order[j], k3);
      last[K3{k3[0], k3[1], k3[2]}] = order[j];  // ascending: the last is the max
    }
    out[h].reserve(last.size());
    for (auto& kv : last) out[h].push_back(kv.second);
  }
  int64_t m = 0;
  for (int h = 0; h < kB; ++h) {
    std::copy(out[h].begin(), out[h].end(), rep_idx + m);
    m += (int64_t)out[h].size();
  }
  std::sort(rep_idx, rep_idx + m);
  *m_out = m;
  return 0;
}

// Reference: estimate_normals (PointCloud.py:68-73), CPUNormals
// (processors.py:243-249).  [upstream] PointCloud::EstimateNormals +
// EstimatePerPointCovariances (Search >= 3 -> ComputeCovariance else
// Identity) + FastEigen3x3; zero -> (0,0,1); prior normals flip the sign.
// normals_out: (n,3) float64.
void oref_estimate_normals(const double* xyz, int64_t n, int mode, int knn, double radius,
                           const double* prior, double* normals_out) {
  std::vector<V3> pts = to_v3(xyz, n);
  KDTree tree;
  tree.build(pts.data(), (int)n);
#pragma omp parallel
  {
    std::vector<int> idx;
    std::vector<double> d2;
#pragma omp for schedule(dynamic, 256)
    for (int64_t i = 0; i < n; ++i) {
      int k = tree.search(pts[i], mode, knn, radius, idx, d2);
      double c[6];
      if (k >= 3) compute_covariance(pts.data(), idx.data(), k, c);
      else {
        c[0] = 1; c[1] = 0; c[2] = 0; c[3] = 1; c[4] = 0; c[5] = 0;
      }
      double nv[3];
      fast_eigen3x3(c, nv);
      double nn = std::sqrt(dot3(nv, nv));
      if (nn == 0.0) {
        if (prior) {
          nv[0] = prior[3 * i]; nv[1] = prior[3 * i + 1]; nv[2] = prior[3 * i + 2];
        } else {
          nv[0] = 0; nv[1] = 0; nv[2] = 1;
        }
      }
      if (prior) {
        double pr[3] = {prior[3 * i], prior[3 * i + 1], prior[3 * i + 2]};
        if (dot3(nv, pr) < 0.0)
          for (int a = 0; a < 3; ++a) nv[a] *= -1.0;
      }
      for (int a = 0; a < 3; ++a) normals_out[3 * i + a] = nv[a];
    }
  }
}

// Batched KDTreeFlann search (PointCloud.py:148-163).  Outputs (nq,K) rows.
void oref_knn_search(const double* xyz, int64_t n, const double* q, int64_t nq, int mode, int knn,
                     double radius, int K, int32_t* idx_out, double* d2_out, int32_t* cnt_out) {
  std::vector<V3> pts = to_v3(xyz, n);
  KDTree tree;
  tree.build(pts.data(), (int)n);
#pragma omp parallel
  {
    std::vector<int> idx;
    std::vector<double> d2;
#pragma omp for schedule(dynamic, 256)
    for (int64_t i = 0; i < nq; ++i) {
      V3 qq{(double)q[3 * i], (double)q[3 * i + 1], (double)q[3 * i + 2]};
      int k = tree.search(qq, mode, knn, radius, idx, d2);
      if (k > K) k = K;
      cnt_out[i] = k;
      for (int j = 0; j < K; ++j) {
        idx_out[i * K + j] = j < k ? idx[j] : -1;
        if (d2_out) d2_out[i * K + j] = j < k ? d2[j] : std::numeric_limits<double>::infinity();
      }
    }
  }
}

// FastEigen3x3 on a batch of covariances {xx,xy,xz,yy,yz,zz} (unit tests).
void oref_fast_eigen3x3(const double* cov, int64_t m, double* out) {
  for (int64_t i = 0; i < m; ++i) fast_eigen3x3(cov + 6 * i, out + 3 * i);
}

// FastEigen3x3 with the transcendental results nudged by one ulp (nudge in
// [0, 27)): the conditioning certificate of the parity tests — a normal that
// moves by more than the tolerance under a 1-ulp acos/cos change is decided
// by the platform's libm, not by the algorithm.
void oref_fast_eigen3x3_nudged(const double* cov, int64_t m, int nudge, double* out) {
  for (int64_t i = 0; i < m; ++i) fast_eigen3x3(cov + 6 * i, out + 3 * i, nudge);
}

// [upstream] utility/Random.cpp + geometry/PointCloudSegmentation.cpp
// RandomSampler: per draw RandUint32() % total, rejected if already in the
// current sample.  Engine: std::mt19937 seeded with `seed`.
void oref_ransac_samples(int64_t n, int ransac_n, int iters, uint64_t seed, int32_t* out) {
  std::mt19937 eng((uint32_t)seed);
  for (int it = 0; it < iters; ++it) {
    int got = 0;
    while (got < ransac_n) {
      int32_t idx = (int32_t)((uint64_t)eng() % (uint64_t)n);
      bool dup = false;
      for (int j = 0; j < got; ++j) dup |= out[it * ransac_n + j] == idx;
      if (!dup) out[it * ransac_n + got++] = idx;
    }
  }
}

// Reference: segment_plane (PointCloud.py:75-77).  [upstream]
// PointCloud::SegmentPlane + EvaluateRANSACBasedOnDistance + GetPlaneFromPoints,
// with the iteration loop replayed sequentially (1 OpenMP thread semantics);
// hypotheses are scored in parallel, which cannot change a hypothesis' score.
// counts/sums (nullable): per-hypothesis inlier count and Sigma|d| (0 for
// degenerate hypotheses, count -1 marks them).  inliers: ascending indices.
int oref_segment_plane(const double* xyz, int64_t n, double thr, int ransac_n, int iters,
                       double prob, const int32_t* samples, double* plane_out, int64_t* inliers,
                       int64_t* n_inliers, int64_t* counts, double* sums, int32_t* best_hyp) {
  if (prob <= 0 || prob > 1) return -22;
  if (ransac_n < 3) return -22;
  if (n < ransac_n) return -22;
  std::vector<V3> pts = to_v3(xyz, n);
  std::vector<double> planes((size_t)iters * 4);
  std::vector<int64_t> cnt(iters);
  std::vector<double> err(iters);
  std::vector<char> degenerate(iters);
  for (int it = 0; it < iters; ++it) {
    double* pl = &planes[(size_t)it * 4];
    if (ransac_n == 3) {
      triangle_plane(pts[samples[it * 3]], pts[samples[it * 3 + 1]], pts[samples[it * 3 + 2]], pl);
    } else {
      std::vector<int64_t> s(ransac_n);
      for (int j = 0; j < ransac_n; ++j) s[j] = samples[it * ransac_n + j];
      plane_from_points(pts.data(), s.data(), ransac_n, pl);
    }
    degenerate[it] = (pl[0] == 0 && pl[1] == 0 && pl[2] == 0 && pl[3] == 0);
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int it = 0; it < iters; ++it) {
    cnt[it] = 0;
    err[it] = 0;
    if (degenerate[it]) continue;
    const double* pl = &planes[(size_t)it * 4];
    double e = 0;
    int64_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
      double d = std::fabs(plane_dist_signed(pl, pts[i]));
      if (d < thr) {
        e += d;
        ++c;
      }
    }
    cnt[it] = c;
    err[it] = e;
  }
  double best_fit = 0, best_rmse = 0;
  int best = -1;
  size_t break_iteration = std::numeric_limits<size_t>::max();
  int iteration_count = 0;
  for (int it = 0; it < iters; ++it) {
    if ((size_t)iteration_count > break_iteration) continue;
    if (degenerate[it]) continue;
    double fit = cnt[it] == 0 ? 0.0 : (double)cnt[it] / (double)n;
    double rmse = cnt[it] == 0 ? 0.0 : err[it] / std::sqrt((double)cnt[it]);
    if (fit > best_fit || (fit == best_fit && rmse < best_rmse)) {
      best_fit = fit;
      best_rmse = rmse;
      best = it;
      if (best_fit < 1.0) {
        double bi = std::min(std::log(1 - prob) / std::log(1 - std::pow(best_fit, ransac_n)), (double)iters);
        break_iteration = (size_t)bi;
      } else {
        break_iteration = 0;
      }
    }
    iteration_count++;
  }
  if (counts)
    for (int it = 0; it < iters; ++it) counts[it] = degenerate[it] ? -1 : cnt[it];
  if (sums)
    for (int it = 0; it < iters; ++it) sums[it] = err[it];
  if (best_hyp) *best_hyp = best;
  double bp[4] = {0, 0, 0, 0};
  if (best >= 0) std::memcpy(bp, &planes[(size_t)best * 4], sizeof(bp));
  int64_t k = 0;
  if (!(bp[0] == 0 && bp[1] == 0 && bp[2] == 0 && bp[3] == 0)) {
    for (int64_t i = 0; i < n; ++i) {
      double d = std::fabs(plane_dist_signed(bp, pts[i]));
      if (d < thr) inliers[k++] = i;
    }
  }
  *n_inliers = k;
  if (k == 0) {
    for (int i = 0; i < 4; ++i) plane_out[i] = 0;
    return 0;
  }
  plane_from_points(pts.data(), inliers, k, plane_out);
  return 0;
}

void oref_plane_from_points(const double* xyz, const int64_t* idx, int64_t k, double* plane_out) {
  // gather the k points as doubles
  std::vector<V3> pts((size_t)k);
  std::vector<int64_t> id((size_t)k);
  for (int64_t j = 0; j < k; ++j) {
    int64_t i = idx[j];
    pts[j] = {(double)xyz[3 * i], (double)xyz[3 * i + 1], (double)xyz[3 * i + 2]};
    id[j] = j;
  }
  plane_from_points(pts.data(), id.data(), k, plane_out);
}

// North-star ICP (no reference symbol).  [upstream]
// pipelines/registration/Registration.cpp RegistrationICP +
// GetRegistrationResultAndCorrespondences (SearchHybrid(p, r, 1)) +
// TransformationEstimation.cpp PointToPlane::ComputeTransformation +
// utility/Eigen.cpp ComputeJTJandJTr / SolveJacobianSystemAndObtainExtrinsicMatrix.
// The source copy is transformed incrementally in float64, as Open3D does.
// corr (nullable, 2*ns int32) / ncorr: final correspondence set.
int oref_registration_icp(const double* src, int64_t ns, const double* tgt, const double* tgt_n,
                          int64_t nt, double max_dist, const double* init, int max_iter,
                          double rel_fit, double rel_rmse, double* T_out, double* fitness,
                          double* rmse, int32_t* corr, int64_t* ncorr) {
  if (max_dist <= 0.0) return -22;
  std::vector<V3> tp = to_v3(tgt, nt);
  std::vector<V3> tn = to_v3(tgt_n, nt);
  std::vector<V3> sp = to_v3(src, ns);
  KDTree tree;
  tree.build(tp.data(), (int)nt);
  double T[16];
  std::memcpy(T, init, sizeof(T));
  bool ident = true;
  for (int i = 0; i < 16; ++i) ident &= T[i] == ((i % 5 == 0) ? 1.0 : 0.0);
  if (!ident) transform_points(T, sp);
  std::vector<int32_t> cj((size_t)ns);
  auto correspond = [&](double& fit, double& rm) -> int64_t {
    double err2 = 0;
    int64_t c = 0;
#pragma omp parallel for reduction(+ : err2, c) schedule(dynamic, 1024)
    for (int64_t i = 0; i < ns; ++i) {
      std::vector<int> idx;
      std::vector<double> d2;
      int k = tree.search(sp[i], 2, 1, max_dist, idx, d2);
      if (k > 0) {
        cj[i] = idx[0];
        err2 += d2[0];
        ++c;
      } else {
        cj[i] = -1;
      }
    }
    if (c == 0) {
      fit = 0;
      rm = 0;
    } else {
      fit = (double)c / (double)ns;
      rm = std::sqrt(err2 / (double)c);
    }
    return c;
  };
  double fit, rm;
  correspond(fit, rm);
  for (int it = 0; it < max_iter; ++it) {
    double JTJ[36] = {0}, JTr[6] = {0};
    for (int64_t i = 0; i < ns; ++i) {
      int j = cj[i];
      if (j < 0) continue;
      const V3& vs = sp[i];
      const V3& vt = tp[j];
      const V3& nt_ = tn[j];
      double d[3] = {vs.x - vt.x, vs.y - vt.y, vs.z - vt.z};
      double nn[3] = {nt_.x, nt_.y, nt_.z};
      double r = dot3(d, nn);
      double vv[3] = {vs.x, vs.y, vs.z};
      double J[6];
      cross(vv, nn, J);
      J[3] = nn[0];
      J[4] = nn[1];
      J[5] = nn[2];
      for (int a = 0; a < 6; ++a) {
        for (int b = 0; b < 6; ++b) JTJ[a * 6 + b] += J[a] * J[b];
        JTr[a] += J[a] * r;
      }
    }
    double upd[16];
    double mb[6];
    for (int a = 0; a < 6; ++a) mb[a] = -JTr[a];
    double x[6];
    bool have_corr = false;
    for (int64_t i = 0; i < ns && !have_corr; ++i) have_corr = cj[i] >= 0;
    if (have_corr && ldlt_solve6(JTJ, mb, x)) vec6_to_mat4(x, upd);
    else {
      for (int a = 0; a < 16; ++a) upd[a] = (a % 5 == 0) ? 1.0 : 0.0;
    }
    mat4_mul(upd, T, T);
    transform_points(upd, sp);
    double pf = fit, pr = rm;
    correspond(fit, rm);
    if (std::fabs(pf - fit) < rel_fit && std::fabs(pr - rm) < rel_rmse) break;
  }
  std::memcpy(T_out, T, sizeof(T));
  *fitness = fit;
  *rmse = rm;
  int64_t k = 0;
  for (int64_t i = 0; i < ns; ++i)
    if (cj[i] >= 0) {
      if (corr) {
        corr[2 * k] = (int32_t)i;
        corr[2 * k + 1] = cj[i];
      }
      ++k;
    }
  *ncorr = k;
  return 0;
}

// Open3D-style single ICP accumulation at transformation T (for sharded tests):
// sums layout = O3DX_ICP_NSUMS (see include/o3dx.h).
void oref_icp_accumulate(const double* src, int64_t ns, const double* tgt, const double* tgt_n,
                         int64_t nt, double max_dist, const double* T, double* sums) {
  std::vector<V3> tp = to_v3(tgt, nt);
  std::vector<V3> tn = to_v3(tgt_n, nt);
  std::vector<V3> sp = to_v3(src, ns);
  transform_points(T, sp);
  KDTree tree;
  tree.build(tp.data(), (int)nt);
  for (int i = 0; i < 32; ++i) sums[i] = 0;
  std::vector<int> idx;
  std::vector<double> d2;
  for (int64_t i = 0; i < ns; ++i) {
    int k = tree.search(sp[i], 2, 1, max_dist, idx, d2);
    if (k == 0) continue;
    const V3& vs = sp[i];
    const V3& vt = tp[idx[0]];
    const V3& nt_ = tn[idx[0]];
    double d[3] = {vs.x - vt.x, vs.y - vt.y, vs.z - vt.z};
    double nn[3] = {nt_.x, nt_.y, nt_.z};
    double r = dot3(d, nn);
    double vv[3] = {vs.x, vs.y, vs.z};
    double J[6];
    cross(vv, nn, J);
    J[3] = nn[0];
    J[4] = nn[1];
    J[5] = nn[2];
    int t = 0;
    for (int a = 0; a < 6; ++a)
      for (int b = a; b < 6; ++b) sums[t++] += J[a] * J[b];
    for (int a = 0; a < 6; ++a) sums[21 + a] += J[a] * r;
    sums[27] += r * r;
    sums[28] += 1.0;
    sums[29] += d2[0];
  }
}

// The exact order-free ("fx") form of the same sums (libo3dx common.hpp /
// include/o3dx.h o3dx_plane_moments note), restated independently for the
// sharded tests: every term rounded to the nearest integer multiple of 2^q
// (ties to even), the integers added in 128 bits.  q per sum from the same
// bounds as icp.hip icp_fx_exps: source |x|,|y|,|z| bounds (absmax), T and
// max_dist.  fx_out: 32 rows {lo = low 32 bits, hi = the rest, q, 0}.
static int fx_exp_of(double B) {
  int e = 0;
  const double b = (B > 0.0 && std::isfinite(B)) ? std::max(B, std::ldexp(1.0, -900)) : 1.0;
  std::frexp(b, &e);
  return e - 51;
}

static void fx_rows(const __int128* acc, const int* q, int k, int64_t* out) {
  for (int j = 0; j < k; ++j) {
    const __int128 v = acc[j];
    const __int128 lo = v & (__int128)0xffffffff;
    out[4 * j] = (int64_t)lo;
    out[4 * j + 1] = (int64_t)((v - lo) / ((__int128)1 << 32));
    out[4 * j + 2] = q[j];
    out[4 * j + 3] = 0;
  }
}

static __int128 fx_int(double t, int q) { return (__int128)std::nearbyint(std::ldexp(t, -q)); }

void oref_icp_accumulate_fx(const double* src, int64_t ns, const double* tgt, const double* tgt_n, int64_t nt,
                            double max_dist, const double* T, const double* absmax, int64_t* fx_out) {
  std::vector<V3> tp = to_v3(tgt, nt);
  std::vector<V3> tn = to_v3(tgt_n, nt);
  std::vector<V3> sp = to_v3(src, ns);
  transform_points(T, sp);
  KDTree tree;
  tree.build(tp.data(), (int)nt);
  int q[32] = {0};
  double P2 = 0.0;
  for (int i = 0; i < 3; ++i) {
    const double Pi = ((std::fabs(T[4 * i]) * absmax[0] + std::fabs(T[4 * i + 1]) * absmax[1]) +
                       std::fabs(T[4 * i + 2]) * absmax[2]) + std::fabs(T[4 * i + 3]);
    P2 += Pi * Pi;
  }
  const double pn = std::sqrt(P2) * 1.01;
  double bJ[6];
  for (int a = 0; a < 6; ++a) bJ[a] = (a < 3 ? pn : 1.0) * 1.01;
  const double br = max_dist * 1.01 * 1.01;
  int t = 0;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) q[t++] = fx_exp_of(bJ[a] * bJ[b] * 1.01);
  for (int a = 0; a < 6; ++a) q[21 + a] = fx_exp_of(bJ[a] * br * 1.01);
  q[27] = fx_exp_of(br * br * 1.01);
  q[28] = fx_exp_of(1.0);
  q[29] = fx_exp_of(max_dist * max_dist * 1.01);
  __int128 acc[32] = {0};
  std::vector<int> idx;
  std::vector<double> d2;
  for (int64_t i = 0; i < ns; ++i) {
    int k = tree.search(sp[i], 2, 1, max_dist, idx, d2);
    if (k == 0) continue;
    const V3& vs = sp[i];
    const V3& vt = tp[idx[0]];
    const V3& nt_ = tn[idx[0]];
    double d[3] = {vs.x - vt.x, vs.y - vt.y, vs.z - vt.z};
    double nn[3] = {nt_.x, nt_.y, nt_.z};
    double r = dot3(d, nn);
    double vv[3] = {vs.x, vs.y, vs.z};
    double J[6];
    cross(vv, nn, J);
    J[3] = nn[0];
    J[4] = nn[1];
    J[5] = nn[2];
    int u = 0;
    for (int a = 0; a < 6; ++a)
      for (int b = a; b < 6; ++b, ++u) acc[u] += fx_int(J[a] * J[b], q[u]);
    for (int a = 0; a < 6; ++a) acc[21 + a] += fx_int(J[a] * r, q[21 + a]);
    acc[27] += fx_int(r * r, q[27]);
    acc[28] += fx_int(1.0, q[28]);
    acc[29] += fx_int(d2[0], q[29]);
  }
  fx_rows(acc, q, 32, fx_out);
}

// host solve from sums (for the sharded CPU test path)
int oref_icp_solve(const double* sums, double* upd) {
  double JTJ[36];
  int t = 0;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) {
      JTJ[a * 6 + b] = sums[t];
      JTJ[b * 6 + a] = sums[t];
      ++t;
    }
  double mb[6], x[6];
  for (int a = 0; a < 6; ++a) mb[a] = -sums[21 + a];
  if (sums[28] <= 0 || !ldlt_solve6(JTJ, mb, x)) {
    for (int a = 0; a < 16; ++a) upd[a] = (a % 5 == 0) ? 1.0 : 0.0;
    return 0;
  }
  vec6_to_mat4(x, upd);
  return 1;
}

}  // extern "C"
