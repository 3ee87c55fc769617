// overlap_probe.hip — calibration microbenchmark (not product code): does a workgroup that
// keeps the NEXT tile's frame loads in flight while it is busy with non-streaming work (main3's
// phases B/C/D) recover the HBM stream that main3 loses?  Each tile: the real C2 decode of 44
// u8 frames (4096 px per 512-lane workgroup), then `spin` shader clocks of non-memory work.
//   mode 0: one tile per workgroup (main3's shape, 2 workgroups per CU)
//   mode 1: persistent workgroups (one per CU, 256 VGPRs), next tile's loads issued before the spin
//   mode 2: persistent workgroups, two per CU, no prefetch (control for the persistence itself)
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/overlap_probe.hip -o /tmp/overlap_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kF = 44, kNC = 11, kNR = 10, kBlock = 512, kPx = 8, kTile = kBlock * kPx;
constexpr int64_t kW = 1920, kH = 1080, kNpx = kW * kH, kStride = (kNpx + 255) / 256 * 256;
constexpr int kTpv = int((kNpx + kTile - 1) / kTile);

typedef unsigned int u32x2e __attribute__((ext_vector_type(2)));

__device__ inline uint32_t gt_u8x4(uint32_t p, uint32_t i) {
  const uint32_t d = (i | 0x80808080u) - (p & 0x7f7f7f7fu);
  return ((p & ~i) | (~(p ^ i) & ~d)) & 0x80808080u;
}
__device__ inline uint32_t gray2bin_x2(uint32_t x) {
  x ^= (x >> 1) & 0x7fff7fffu; x ^= (x >> 2) & 0x3fff3fffu;
  x ^= (x >> 4) & 0x0fff0fffu; x ^= (x >> 8) & 0x00ff00ffu;
  return x;
}
__device__ inline uint2 ld8(const uint8_t* a) {
  const u32x2e e = __builtin_nontemporal_load(reinterpret_cast<const u32x2e*>(a));
  return make_uint2(e.x, e.y);
}

struct Stack { uint2 v[kF]; };

__device__ inline void issue(Stack& s, const uint8_t* frames, int64_t vb, int t) {
  const int view = t % 12, tile = t / 12;
  int64_t px0 = int64_t(tile) * kTile + int64_t(threadIdx.x) * kPx;
  if (px0 >= kNpx) px0 = 0;
  const uint8_t* f = frames + view * vb + px0;
#pragma unroll
  for (int fr = 0; fr < kF; ++fr) s.v[fr] = ld8(f + fr * kStride);
}

__device__ inline uint32_t consume(const Stack& s) {
  uint32_t ac[4] = {}, ar[4] = {};
#pragma unroll
  for (int b = 0; b < kNC; ++b)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t m = gt_u8x4(k ? s.v[2 + 2 * b].y : s.v[2 + 2 * b].x, k ? s.v[3 + 2 * b].y : s.v[3 + 2 * b].x);
      ac[2 * k] = (ac[2 * k] << 1) | ((m >> 7) & 0x00010001u);
      ac[2 * k + 1] = (ac[2 * k + 1] << 1) | ((m >> 15) & 0x00010001u);
    }
#pragma unroll
  for (int b = 0; b < kNR; ++b)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t m = gt_u8x4(k ? s.v[24 + 2 * b].y : s.v[24 + 2 * b].x, k ? s.v[25 + 2 * b].y : s.v[25 + 2 * b].x);
      ar[2 * k] = (ar[2 * k] << 1) | ((m >> 7) & 0x00010001u);
      ar[2 * k + 1] = (ar[2 * k + 1] << 1) | ((m >> 15) & 0x00010001u);
    }
  uint32_t h = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) h += gray2bin_x2(ac[j]) * 3u + gray2bin_x2(ar[j]);
  h ^= __builtin_amdgcn_perm(s.v[0].x, s.v[1].y, 0x05010400u);
  return h;
}

// non-memory work of ~`spin` shader clocks (the look-back wait and fp64 chain stand-in)
__device__ inline uint32_t busy(uint32_t h, uint32_t spin) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < spin) {
#pragma unroll
    for (int k = 0; k < 16; ++k) h = h * 2654435761u + 0x9e3779b9u;
  }
  return h;
}

__global__ __launch_bounds__(kBlock, 4) void tile_kernel(const uint8_t* frames, int64_t vb, uint32_t spin, uint32_t* sink) {
  Stack s;
  issue(s, frames, vb, blockIdx.x);
  uint32_t h = consume(s);
  __syncthreads();
  h = busy(h, spin);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sink[blockIdx.x & 1023] = h;
}

template <int WAVES>
__global__ __launch_bounds__(kBlock, WAVES) void persist_kernel(const uint8_t* frames, int64_t vb, uint32_t spin,
                                                               int n_tiles, int prefetch, uint32_t* sink) {
  Stack s;
  int t = blockIdx.x;
  uint32_t h = 0;
  if (t < n_tiles) issue(s, frames, vb, t);
  for (; t < n_tiles; t += gridDim.x) {
    h += consume(s);
    __syncthreads();
    const int tn = t + gridDim.x;
    if (prefetch && tn < n_tiles) issue(s, frames, vb, tn);
    h = busy(h, spin);
    __syncthreads();
    if (!prefetch && tn < n_tiles) issue(s, frames, vb, tn);
  }
  if ((threadIdx.x & 63) == 0) sink[blockIdx.x & 1023] = h;
}

__global__ void fill(uint8_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n / 4; i += int64_t(gridDim.x) * blockDim.x) {
    uint32_t x = uint32_t(i) * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    reinterpret_cast<uint32_t*>(p)[i] = x;
  }
}

int main() {
  const int n_views = 12, n_tiles = kTpv * n_views;
  const int64_t vb = int64_t(kF) * kStride + 64 * 4096;
  uint8_t* frames; uint32_t* sink;
  CK(hipMalloc(&frames, vb * n_views));
  CK(hipMalloc(&sink, 4096 * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, frames, vb * n_views, 7u);
  CK(hipDeviceSynchronize());
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto time = [&](const char* name, uint32_t spin, auto launch) {
    std::vector<float> ts;
    for (int it = 0; it < 30; ++it) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (it >= 4) ts.push_back(ms * 1e3f / n_views);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    printf("%-40s spin %6u  %7.2f us/view  %6.0f GB/s\n", name, spin, us, double(kF) * kNpx / us / 1e3);
    fflush(stdout);
  };
  for (uint32_t spin : {0u, 5000u, 10000u, 20000u, 30000u}) {
    time("tile/workgroup (main3 shape)", spin, [&] {
      hipLaunchKernelGGL(tile_kernel, dim3(n_tiles), dim3(kBlock), 0, 0, frames, vb, spin, sink);
    });
    time("persistent 2/CU, no prefetch", spin, [&] {
      hipLaunchKernelGGL(persist_kernel<4>, dim3(2 * cus), dim3(kBlock), 0, 0, frames, vb, spin, n_tiles, 0, sink);
    });
    time("persistent 2/CU, prefetch", spin, [&] {
      hipLaunchKernelGGL(persist_kernel<4>, dim3(2 * cus), dim3(kBlock), 0, 0, frames, vb, spin, n_tiles, 1, sink);
    });
    time("persistent 1/CU, prefetch", spin, [&] {
      hipLaunchKernelGGL(persist_kernel<2>, dim3(cus), dim3(kBlock), 0, 0, frames, vb, spin, n_tiles, 1, sink);
    });
  }
  return 0;
}
