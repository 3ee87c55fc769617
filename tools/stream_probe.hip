// stream_probe.hip — calibration microbenchmark (not product code): how fast can the decode
// phase stream a C2 frame stack (44 u8 frames of 1920x1080) on MI355X, by load width, pixels
// per lane, tile geometry, loads in flight, and views per launch.  Each variant does the real
// per-pixel decode work (strict byte compares, bit pack, Gray->binary, integer mask) and folds
// the result into one word per workgroup so nothing is dead-code eliminated.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/stream_probe.hip -o /tmp/stream_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kF = 44, kNC = 11, kNR = 10;
constexpr int64_t kW = 1920, kH = 1080, kNpx = kW * kH, kStride = (kNpx + 255) / 256 * 256;

__device__ inline uint32_t gt_u8x4(uint32_t p, uint32_t i) {
  const uint32_t d = (i | 0x80808080u) - (p & 0x7f7f7f7fu);
  return ((p & ~i) | (~(p ^ i) & ~d)) & 0x80808080u;
}
__device__ inline uint32_t gray2bin_x2(uint32_t x) {
  x ^= (x >> 1) & 0x7fff7fffu; x ^= (x >> 2) & 0x3fff3fffu;
  x ^= (x >> 4) & 0x0fff0fffu; x ^= (x >> 8) & 0x00ff00ffu;
  return x;
}
__device__ inline void acc4(uint32_t (&a)[4], uint32_t p, uint32_t i, int j) {
  const uint32_t m = gt_u8x4(p, i);
  a[2 * j] = (a[2 * j] << 1) | ((m >> 7) & 0x00010001u);
  a[2 * j + 1] = (a[2 * j + 1] << 1) | ((m >> 15) & 0x00010001u);
}

template <int W>  // load width in dwords: 2 (8 B) or 4 (16 B)
struct Vec;
typedef unsigned int u32x2e __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));
template <> struct Vec<2> { using T = uint2; using E = u32x2e; };
template <> struct Vec<4> { using T = uint4; using E = u32x4e; };

__device__ inline uint32_t getw(const uint2& v, int k) { return k == 0 ? v.x : v.y; }
__device__ inline uint32_t getw(const uint4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// One lane decodes PX = 4*W pixels; loads of BATCH (col,row) pair groups are issued together.
// LAYOUT 0: frame-major [view][frame][stride] (the product layout); 1: tile-interleaved
// [view][tile][frame][TILE] (one contiguous 44*TILE run per workgroup).  NT: non-temporal loads.
template <int W, int BATCH, int BLOCK, int LAYOUT = 0, int NT = 0, int STORE = 0>
__global__ __launch_bounds__(BLOCK) void probe(const uint8_t* frames, int64_t view_bytes, int tiles_per_view,
                                               uint32_t* sink, float* xyz, uint8_t* bgr) {
  using V = typename Vec<W>::T;
  constexpr int PX = 4 * W;
  constexpr int TILE = BLOCK * PX;
  const int view = blockIdx.x / tiles_per_view, tile = blockIdx.x - view * tiles_per_view;
  const uint8_t* f = frames + view * view_bytes;
  int64_t px0 = int64_t(tile) * TILE + int64_t(threadIdx.x) * PX;
  if (px0 >= kNpx) px0 = 0;
  const int64_t tb = int64_t(tile) * kF * TILE + int64_t(threadIdx.x) * PX;
  auto ld = [&](int fr) {
    const uint8_t* a = LAYOUT ? f + tb + fr * TILE : f + fr * kStride + px0;
    if constexpr (NT) {
      const typename Vec<W>::E e = __builtin_nontemporal_load(reinterpret_cast<const typename Vec<W>::E*>(a));
      V v;
      __builtin_memcpy(&v, &e, sizeof(v));
      return v;
    } else {
      return *reinterpret_cast<const V*>(a);
    }
  };
  const V w = ld(0), b = ld(1);
  uint32_t ac[2 * W] = {}, ar[2 * W] = {};
#pragma unroll
  for (int b0 = 0; b0 < kNC; b0 += BATCH) {
    V cp[BATCH], ci[BATCH], rp[BATCH], ri[BATCH];
#pragma unroll
    for (int g = 0; g < BATCH; ++g) if (b0 + g < kNC) { cp[g] = ld(2 + 2 * (b0 + g)); ci[g] = ld(3 + 2 * (b0 + g)); }
#pragma unroll
    for (int g = 0; g < BATCH; ++g) if (b0 + g < kNR) { rp[g] = ld(24 + 2 * (b0 + g)); ri[g] = ld(25 + 2 * (b0 + g)); }
#pragma unroll
    for (int g = 0; g < BATCH; ++g) if (b0 + g < kNC) {
#pragma unroll
      for (int k = 0; k < W; ++k) {
        uint32_t t[4] = {ac[0], ac[1], 0, 0};
        (void)t;
        const uint32_t m = gt_u8x4(getw(cp[g], k), getw(ci[g], k));
        ac[2 * k] = (ac[2 * k] << 1) | ((m >> 7) & 0x00010001u);
        ac[2 * k + 1] = (ac[2 * k + 1] << 1) | ((m >> 15) & 0x00010001u);
      }
    }
#pragma unroll
    for (int g = 0; g < BATCH; ++g) if (b0 + g < kNR) {
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const uint32_t m = gt_u8x4(getw(rp[g], k), getw(ri[g], k));
        ar[2 * k] = (ar[2 * k] << 1) | ((m >> 7) & 0x00010001u);
        ar[2 * k + 1] = (ar[2 * k + 1] << 1) | ((m >> 15) & 0x00010001u);
      }
    }
  }
  uint32_t h = 0;
#pragma unroll
  for (int j = 0; j < 2 * W; ++j) h += gray2bin_x2(ac[j]) * 3u + gray2bin_x2(ar[j]);
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const uint32_t wv = getw(w, k), bv = getw(b, k);
    h ^= __builtin_amdgcn_perm(wv, bv, 0x05010400u) + (wv > 0x40404040u);
  }
  if constexpr (STORE) {
    // the cloud of this tile: 57 % of its pixels (the C2 bench's valid fraction), compacted
    // points at consecutive addresses, one point per lane per round (as main3 phase D)
    constexpr int TILE = BLOCK * 4 * W;
    const int64_t base = int64_t(blockIdx.x) * (TILE * 57 / 100);
    for (int i = threadIdx.x; i < TILE * 57 / 100; i += BLOCK) {
      const int64_t q = base + i;
      if constexpr (STORE == 1) {
        xyz[3 * q] = float(h); xyz[3 * q + 1] = float(h + 1); xyz[3 * q + 2] = float(h + 2);
        bgr[3 * q] = uint8_t(h); bgr[3 * q + 1] = uint8_t(h >> 8); bgr[3 * q + 2] = uint8_t(h >> 16);
      } else {
        reinterpret_cast<uint4*>(xyz)[q] = make_uint4(h, h + 1, h + 2, h + 3);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(sink + (blockIdx.x & 1023), h);
}

__global__ void fill(uint8_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n / 4; i += int64_t(gridDim.x) * blockDim.x) {
    uint32_t x = uint32_t(i) * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    reinterpret_cast<uint32_t*>(p)[i] = x;
  }
}

template <int W, int BATCH, int BLOCK, int LAYOUT = 0, int NT = 0, int STORE = 0>
void run(const char* name, const uint8_t* frames, int n_views, int views_per_launch, uint32_t* sink,
         float* xyz = nullptr, uint8_t* bgr = nullptr) {
  constexpr int TILE = BLOCK * 4 * W;
  const int tpv = int((kNpx + TILE - 1) / TILE);
  const int64_t vb = int64_t(kF) * kStride + 64 * 4096;  // room for the interleaved tail tile
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int it = 0; it < 40; ++it) {
    const int v0 = (it * views_per_launch) % n_views;
    const int nv = std::min(views_per_launch, n_views - v0);
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((probe<W, BATCH, BLOCK, LAYOUT, NT, STORE>), dim3(tpv * nv), dim3(BLOCK), 0, 0, frames + v0 * vb, vb, tpv, sink, xyz, bgr);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 4) ts.push_back(ms * 1e3f / nv);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[ts.size() / 2];
  printf("%-34s views/launch %d  %7.2f us/view  %6.0f GB/s\n", name, views_per_launch, us, double(kF) * kNpx / us / 1e3);
}

int main() {
  const int n_views = 12;
  const int64_t vb = int64_t(kF) * kStride + 64 * 4096;
  uint8_t* frames; uint32_t* sink;
  CK(hipMalloc(&frames, vb * n_views));
  CK(hipMalloc(&sink, 4096 * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, frames, vb * n_views, 7u);
  CK(hipDeviceSynchronize());
  float* xyz; uint8_t* bgr;
  CK(hipMalloc(&xyz, int64_t(n_views) * kNpx * 16));
  CK(hipMalloc(&bgr, int64_t(n_views) * kNpx * 3));
  for (int vpl : {12}) {
    run<2, 11, 256, 0, 1>("u2 8px batch11 frame-major nt", frames, n_views, vpl, sink);
    run<2, 11, 256, 0, 1, 1>("  + cloud stores (12 B + 3 B)", frames, n_views, vpl, sink, xyz, bgr);
    run<2, 11, 256, 0, 1, 2>("  + cloud stores (16-B records)", frames, n_views, vpl, sink, xyz, bgr);
    run<2, 11, 512, 0, 1>("u2 8px batch11 blk512 nt", frames, n_views, vpl, sink);
    run<2, 11, 512, 0, 1, 1>("  + cloud stores (12 B + 3 B)", frames, n_views, vpl, sink, xyz, bgr);
    run<2, 11, 256, 0, 1>("u2 8px batch11 frame-major nt (again)", frames, n_views, vpl, sink);
  }
  return 0;
}
