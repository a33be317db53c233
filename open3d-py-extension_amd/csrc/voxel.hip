// voxel.hip — voxel down-sample with trace.
//
// Replaces o3d PointCloud.voxel_down_sample_and_trace(vs, min_bound, max_bound,
// approximate_class=False) + idxmat.max(1) + _select_by_idx
// (reference open3dpypro/PointCloud.py:338-341, :361-362, :185-204;
// processors.py:427-430 VoxelDownsample.cpu_model).
//
// Layout & algorithm (HBM-bound integer work; no MFMA):
//   1. key per point in float64 exactly as Open3D: floor(((double)p - min)/vs).
//   2. voxel table: dense int32 array over the grid box when it is small
//      (<= 2n + 2^20 cells), else an open-addressing hash table on a packed
//      63-bit key.  rep[voxel] = atomicMax(point index)  (= idxmat.max(1)).
//   3. flags[rep] = 1, then a flag compaction gives the representatives in
//      ascending index order (= _select_by_idx order) for free.
//   4. trace (optional): voxel_of_point via the compaction prefix, Open3D's
//      (M,8) cubic-id matrix via atomicMax into octant slots.
#include "common.hpp"

namespace o3dx {

constexpr uint64_t kEmpty = ~0ull;
constexpr int kHashBits = 21;
constexpr int kHashOff = 1 << (kHashBits - 1);

struct VoxelGeom {
  double mnx, mny, mnz, vs;
  int nx, ny, nz;
};

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

struct P3 {
  float x, y, z;
};

// Open3D: ref_coord = (p - voxel_min_bound) / voxel_size; voxel_index = floor.
__device__ __forceinline__ void voxel_ref(const P3& q, const VoxelGeom& g, double r[3], int v[3]) {
  r[0] = ((double)q.x - g.mnx) / g.vs;
  r[1] = ((double)q.y - g.mny) / g.vs;
  r[2] = ((double)q.z - g.mnz) / g.vs;
  v[0] = (int)floor(r[0]);
  v[1] = (int)floor(r[1]);
  v[2] = (int)floor(r[2]);
}

__global__ void __launch_bounds__(kBlock) k_voxel_assign_dense(const float* __restrict__ xyz, int64_t n,
                                                               VoxelGeom g, int32_t* __restrict__ rep,
                                                               int32_t* __restrict__ vid, int* __restrict__ err) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double r[3];
    int v[3];
    voxel_ref(p[i], g, r, v);
    if (v[0] < 0 || v[0] >= g.nx || v[1] < 0 || v[1] >= g.ny || v[2] < 0 || v[2] >= g.nz) {
      *err = 1;
      vid[i] = -1;
      continue;
    }
    int32_t id = v[0] + g.nx * (v[1] + g.ny * v[2]);
    vid[i] = id;
    rep[id] = (int32_t)i;  // plain store: some index of the voxel wins (k_voxel_settle makes it the max)
  }
}

// Second half of the dense assignment: the racy plain stores above left one of
// each voxel's indices in the table; only points with a larger index need the
// (device-scope, slow) atomicMax.  Grid-stride rounds run in index order, so
// the last writer usually is already the maximum and few atomics remain.
__global__ void __launch_bounds__(kBlock) k_voxel_settle(const int32_t* __restrict__ vid, int64_t n,
                                                         int32_t* __restrict__ rep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t id = vid[i];
    if (id >= 0 && rep[id] < (int32_t)i) atomicMax(&rep[id], (int32_t)i);
  }
}

__global__ void __launch_bounds__(kBlock) k_voxel_assign_hash(const float* __restrict__ xyz, int64_t n,
                                                              VoxelGeom g, unsigned long long* __restrict__ keys,
                                                              int32_t* __restrict__ rep, uint32_t tmask,
                                                              int32_t* __restrict__ vid, int* __restrict__ err) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double r[3];
    int v[3];
    voxel_ref(p[i], g, r, v);
    bool bad = false;
    uint64_t key = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      int o = v[a] + kHashOff;
      bad |= (o < 0) | (o >= (1 << kHashBits));
      key |= (uint64_t)(uint32_t)o << (kHashBits * a);
    }
    if (bad) {
      *err = 2;
      vid[i] = 0;
      continue;
    }
    uint32_t s = (uint32_t)mix64(key) & tmask;
    while (true) {
      unsigned long long prev = atomicCAS(&keys[s], (unsigned long long)kEmpty, (unsigned long long)key);
      if (prev == kEmpty || prev == key) break;
      s = (s + 1) & tmask;
    }
    vid[i] = (int32_t)s;
    atomicMax(&rep[s], (int32_t)i);
  }
}

__global__ void __launch_bounds__(kBlock) k_voxel_mark(const int32_t* __restrict__ rep, int64_t nslots,
                                                       uint8_t* __restrict__ flags) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nslots; v += (int64_t)gridDim.x * blockDim.x) {
    int32_t r = rep[v];
    if (r >= 0) flags[r] = 1;
  }
}

__global__ void __launch_bounds__(kBlock) k_gather_xyz(const float* __restrict__ xyz, const int32_t* __restrict__ idx,
                                                       int64_t m, float* __restrict__ out) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  P3* o = reinterpret_cast<P3*>(out);
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
    o[j] = p[idx[j]];
}

__global__ void __launch_bounds__(kBlock) k_voxel_trace(const float* __restrict__ xyz, int64_t n, VoxelGeom g,
                                                        const int32_t* __restrict__ vid,
                                                        const int32_t* __restrict__ rep,
                                                        const int32_t* __restrict__ pos,
                                                        int32_t* __restrict__ voxel_of_point,
                                                        int32_t* __restrict__ cubic) {
  const P3* p = reinterpret_cast<const P3*>(xyz);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t row = pos[rep[vid[i]]];
    if (voxel_of_point) voxel_of_point[i] = row;
    if (cubic) {
      double r[3];
      int v[3];
      voxel_ref(p[i], g, r, v);
      // Open3D: cid += {1,2,4}[c] when (ref_coord(c) - voxel_index(c)) >= 0.5
      int cid = ((r[0] - v[0]) >= 0.5 ? 1 : 0) + ((r[1] - v[1]) >= 0.5 ? 2 : 0) + ((r[2] - v[2]) >= 0.5 ? 4 : 0);
      atomicMax(&cubic[(int64_t)row * 8 + cid], (int32_t)i);
    }
  }
}

static int64_t dense_cap(int64_t n) { return 2 * n + (1 << 20); }
static int64_t hash_cap(int64_t n) {
  int64_t t = 1024;
  while (t < 2 * n) t <<= 1;
  return t;
}

struct VoxelWs {
  int32_t* table;              // dense rep or hash rep
  unsigned long long* keys;    // hash keys
  int32_t* vid;
  uint8_t* flags;
  int32_t* pos;
  int32_t* scan_tmp;
  char* aabb;
  double* mm;
  int64_t* count;  // [0] = m, [1] = err (as int)
};

static size_t carve(Arena& ar, int64_t n, VoxelWs* w) {
  int64_t dc = dense_cap(n), hc = hash_cap(n);
  // one region shared by the dense table or the hash (keys + rep)
  size_t table_bytes = std::max<size_t>(dc * sizeof(int32_t), hc * (sizeof(int32_t) + sizeof(uint64_t)));
  char* tb = ar.take<char>(table_bytes);
  w->table = reinterpret_cast<int32_t*>(tb);
  w->keys = tb ? reinterpret_cast<unsigned long long*>(tb + Arena::align(hc * sizeof(int32_t))) : nullptr;
  w->vid = ar.take<int32_t>(n);
  w->flags = ar.take<uint8_t>(n + 16);
  w->pos = ar.take<int32_t>(n);
  w->scan_tmp = ar.take<int32_t>(compact_workspace_ints(n));
  w->aabb = ar.take<char>(aabb_ws_bytes(n));
  w->mm = ar.take<double>(8);
  w->count = ar.take<int64_t>(4);
  return ar.used;
}

}  // namespace o3dx

using namespace o3dx;

extern "C" size_t o3dx_voxel_workspace_bytes(int64_t n) {
  Arena ar(nullptr, 0);
  VoxelWs w;
  // hash keys live after an aligned rep block inside the table region
  return carve(ar, std::max<int64_t>(n, 1), &w) + Arena::align(hash_cap(std::max<int64_t>(n, 1)) * 4) + 1024;
}

extern "C" int o3dx_voxel_down_sample(const float* xyz, int64_t n, const double* min_bound_host,
                                      const double* max_bound_host, double voxel_size, int32_t* rep_idx,
                                      float* rep_xyz, int64_t* m_host, int32_t* voxel_of_point, int32_t* cubic_id,
                                      void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !rep_idx)) || !m_host)
    return fail(O3DX_EINVAL, "o3dx_voxel_down_sample: bad arguments");
  if (!(voxel_size > 0.0)) return fail(O3DX_EINVAL, "voxel_size <= 0.");
  if (ws_bytes < o3dx_voxel_workspace_bytes(n) || !ws)
    return fail(O3DX_ENOMEM, "o3dx_voxel_down_sample: workspace too small (need %zu)", o3dx_voxel_workspace_bytes(n));
  hipStream_t s = as_stream(stream);
  Arena ar(ws, ws_bytes);
  VoxelWs w;
  carve(ar, std::max<int64_t>(n, 1), &w);
  w.keys = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w.table) +
                                                 Arena::align(hash_cap(std::max<int64_t>(n, 1)) * 4));

  double mn[3], mx[3];
  if (!min_bound_host || !max_bound_host) {
    double mm[6];
    O3DX_TRY(aabb_device(xyz, n, w.mm, w.aabb, s));
    O3DX_HIP(hipMemcpyAsync(mm, w.mm, 6 * sizeof(double), hipMemcpyDeviceToHost, s));
    O3DX_HIP(hipStreamSynchronize(s));
    for (int a = 0; a < 3; ++a) {
      mn[a] = min_bound_host ? min_bound_host[a] : mm[a];
      mx[a] = max_bound_host ? max_bound_host[a] : mm[3 + a];
    }
  } else {
    for (int a = 0; a < 3; ++a) {
      mn[a] = min_bound_host[a];
      mx[a] = max_bound_host[a];
    }
  }
  // Open3D: if (voxel_size * INT_MAX < (max_bound - min_bound).maxCoeff()) LogError
  double ext = std::max(mx[0] - mn[0], std::max(mx[1] - mn[1], mx[2] - mn[2]));
  if (voxel_size * (double)INT32_MAX < ext) return fail(O3DX_EINVAL, "voxel_size is too small.");
  if (n == 0) {
    *m_host = 0;
    return 0;
  }
  VoxelGeom g;
  g.mnx = mn[0];
  g.mny = mn[1];
  g.mnz = mn[2];
  g.vs = voxel_size;
  double dims[3];
  for (int a = 0; a < 3; ++a) dims[a] = std::floor(std::max(0.0, mx[a] - mn[a]) / voxel_size) + 1.0;
  double nvox = dims[0] * dims[1] * dims[2];
  bool dense = nvox <= (double)dense_cap(n);
  g.nx = (int)dims[0];
  g.ny = (int)dims[1];
  g.nz = (int)dims[2];

  const unsigned grid = grid_for(n, kBlock, 8192);
  int64_t counts[2];
  for (int attempt = 0; attempt < 2; ++attempt) {
    int64_t nslots;
    O3DX_HIP(hipMemsetAsync(w.count, 0, 4 * sizeof(int64_t), s));
    if (dense) {
      nslots = (int64_t)nvox;
      O3DX_HIP(hipMemsetAsync(w.table, 0xFF, nslots * sizeof(int32_t), s));
      KTimer kt("voxel_assign", s);
      hipLaunchKernelGGL(k_voxel_assign_dense, dim3(grid), dim3(kBlock), 0, s, xyz, n, g, w.table, w.vid,
                         reinterpret_cast<int*>(w.count + 1));
      hipLaunchKernelGGL(k_voxel_settle, dim3(grid), dim3(kBlock), 0, s, w.vid, n, w.table);
    } else {
      nslots = hash_cap(n);
      O3DX_HIP(hipMemsetAsync(w.table, 0xFF, nslots * sizeof(int32_t), s));
      O3DX_HIP(hipMemsetAsync(w.keys, 0xFF, nslots * sizeof(uint64_t), s));
      KTimer kt("voxel_assign", s);
      hipLaunchKernelGGL(k_voxel_assign_hash, dim3(grid), dim3(kBlock), 0, s, xyz, n, g, w.keys, w.table,
                         (uint32_t)(nslots - 1), w.vid, reinterpret_cast<int*>(w.count + 1));
    }
    {
      KTimer kt("voxel_compact", s);
      O3DX_HIP(hipMemsetAsync(w.flags, 0, n, s));
      hipLaunchKernelGGL(k_voxel_mark, dim3(grid_for(nslots, kBlock, 8192)), dim3(kBlock), 0, s, w.table, nslots,
                         w.flags);
      O3DX_TRY(compact_flags(w.flags, n, rep_idx, (voxel_of_point || cubic_id) ? w.pos : nullptr, w.count,
                             w.scan_tmp, s));
    }
    O3DX_HIP(hipMemcpyAsync(counts, w.count, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    O3DX_HIP(hipStreamSynchronize(s));
    int errflag = (int)(counts[1] & 0xffffffff);
    if (errflag == 0) break;
    if (errflag == 2 || !dense)
      return fail(O3DX_ENOTSUP, "voxel grid spans more than 2^%d cells per axis", kHashBits);
    dense = false;  // points outside the given bounds: retry with the hash table
  }
  const int64_t m = counts[0];
  *m_host = m;
  if (rep_xyz && m > 0)
    hipLaunchKernelGGL(k_gather_xyz, dim3(grid_for(m, kBlock, 8192)), dim3(kBlock), 0, s, xyz, rep_idx, m, rep_xyz);
  if ((voxel_of_point || cubic_id) && m > 0) {
    if (cubic_id) O3DX_HIP(hipMemsetAsync(cubic_id, 0xFF, (size_t)m * 8 * sizeof(int32_t), s));
    hipLaunchKernelGGL(k_voxel_trace, dim3(grid), dim3(kBlock), 0, s, xyz, n, g, w.vid, w.table, w.pos,
                       voxel_of_point, cubic_id);
  }
  O3DX_HIP(hipGetLastError());
  return 0;
}
