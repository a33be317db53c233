// pcd.hip — PCD (Point Cloud Data) field decoding on the device.
//
// Replaces the per-field host decoding of o3d.io.read_point_cloud behind
// PointCloudBase.read_pcd (reference open3dpypro/PointCloud.py:165-166).  The
// host parses the header, moves the raw DATA bytes (binary records, or the
// LZF-decompressed column blocks of binary_compressed) to HBM once; this
// kernel converts every field of every point in one pass: byte-exact reads
// (records need not be aligned), conversion to float32, and the packed
// 0x00RRGGBB colour split into r, g, b in [0, 1].  Byte work, HBM bound.
#include <cstring>

#include "common.hpp"

namespace o3dx {

constexpr int kPcdMaxFields = 16;

struct PcdFields {
  int nf;
  int type[kPcdMaxFields];
  int64_t src_off[kPcdMaxFields];
  int64_t src_stride[kPcdMaxFields];
  float* dst[kPcdMaxFields];
  int64_t dst_stride[kPcdMaxFields];
};

template <class T>
__device__ __forceinline__ T load_unaligned(const uint8_t* p) {
  T v;
  __builtin_memcpy(&v, p, sizeof(T));
  return v;
}

__global__ void __launch_bounds__(kBlock) k_pcd_unpack(const uint8_t* __restrict__ data, int64_t n, PcdFields f) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    for (int j = 0; j < f.nf; ++j) {
      const uint8_t* p = data + f.src_off[j] + i * f.src_stride[j];
      float* d = f.dst[j] + i * f.dst_stride[j];
      switch (f.type[j]) {
        case O3DX_PCD_F4: d[0] = load_unaligned<float>(p); break;
        case O3DX_PCD_F8: d[0] = (float)load_unaligned<double>(p); break;
        case O3DX_PCD_U1: d[0] = (float)load_unaligned<uint8_t>(p); break;
        case O3DX_PCD_U2: d[0] = (float)load_unaligned<uint16_t>(p); break;
        case O3DX_PCD_U4: d[0] = (float)load_unaligned<uint32_t>(p); break;
        case O3DX_PCD_I1: d[0] = (float)load_unaligned<int8_t>(p); break;
        case O3DX_PCD_I2: d[0] = (float)load_unaligned<int16_t>(p); break;
        case O3DX_PCD_I4: d[0] = (float)load_unaligned<int32_t>(p); break;
        case O3DX_PCD_RGB: {
          const uint32_t u = load_unaligned<uint32_t>(p);
          d[0] = (float)((u >> 16) & 0xFFu) / 255.0f;
          d[1] = (float)((u >> 8) & 0xFFu) / 255.0f;
          d[2] = (float)(u & 0xFFu) / 255.0f;
          break;
        }
        default: break;
      }
    }
  }
}

}  // namespace o3dx

using namespace o3dx;

// liblzf decompression (PCD DATA binary_compressed), host side: the stream is
// sequential, so it runs on the CPU before the single host-to-device copy.
extern "C" int64_t o3dx_lzf_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t dst_len) {
  if (n < 0 || dst_len < 0 || (n > 0 && !src) || (dst_len > 0 && !dst)) return fail(O3DX_EINVAL, "lzf: bad arguments");
  int64_t ip = 0, op = 0;
  while (ip < n) {
    const unsigned ctrl = src[ip++];
    if (ctrl < 32) {  // literal run of ctrl + 1 bytes
      const int64_t len = ctrl + 1;
      if (ip + len > n || op + len > dst_len) return fail(O3DX_EINVAL, "lzf: corrupt stream (literal)");
      std::memcpy(dst + op, src + ip, (size_t)len);
      ip += len;
      op += len;
    } else {  // back reference, may overlap
      int64_t len = ctrl >> 5;
      int64_t ref = op - ((int64_t)(ctrl & 0x1f) << 8) - 1;
      if (len == 7) {
        if (ip >= n) return fail(O3DX_EINVAL, "lzf: corrupt stream (length)");
        len += src[ip++];
      }
      if (ip >= n) return fail(O3DX_EINVAL, "lzf: corrupt stream (offset)");
      ref -= src[ip++];
      len += 2;
      if (ref < 0 || op + len > dst_len) return fail(O3DX_EINVAL, "lzf: corrupt stream (reference)");
      for (int64_t k = 0; k < len; ++k) dst[op + k] = dst[ref + k];
      op += len;
    }
  }
  return op;
}

extern "C" int o3dx_pcd_unpack(const uint8_t* data, int64_t n, int nfields, const int32_t* types,
                               const int64_t* src_off, const int64_t* src_stride, float* const* dst,
                               const int64_t* dst_stride, void* stream) {
  if (n < 0 || nfields < 0 || nfields > kPcdMaxFields || (n > 0 && nfields > 0 && !data))
    return fail(O3DX_EINVAL, "o3dx_pcd_unpack: bad arguments");
  if (n == 0 || nfields == 0) return 0;
  if (!types || !src_off || !src_stride || !dst || !dst_stride) return fail(O3DX_EINVAL, "o3dx_pcd_unpack: null field table");
  PcdFields f;
  f.nf = nfields;
  for (int j = 0; j < nfields; ++j) {
    if (types[j] < O3DX_PCD_F4 || types[j] > O3DX_PCD_RGB || !dst[j] || src_off[j] < 0 || src_stride[j] < 0)
      return fail(O3DX_EINVAL, "o3dx_pcd_unpack: bad field %d", j);
    f.type[j] = types[j];
    f.src_off[j] = src_off[j];
    f.src_stride[j] = src_stride[j];
    f.dst[j] = dst[j];
    f.dst_stride[j] = dst_stride[j];
  }
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_pcd_unpack, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, data, n, f);
  O3DX_HIP(hipGetLastError());
  return 0;
}
