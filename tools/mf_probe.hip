// mf_probe.hip — calibration microbenchmark (not product code): what a mask-first decode of a
// C2 frame stack (44 u8 frames of 1920x1080) can stream on MI355X when only the lanes holding a
// valid pixel read the 42 pattern frames.  The mask is a real rendered view's (tools/mf_probe.py
// writes it: one byte per pixel); frame 0 holds 255 / 0 by it, frame 1 zeros, the pattern frames
// random bytes.  Variants:
//   dense    every lane reads every frame (main3 before the mask-first change)
//   mf       white/black first, pattern loads only in lanes with a valid pixel (main3 now)
//   mf_l2    the lane's decision from a per-lane byte table that every view shares (L2-resident):
//            the same bytes as mf, the dependent round trip at L2 instead of HBM latency
//   mf16     mf with 16 px per lane (16-byte loads), half the load instructions
// Each variant does the SWAR decode and folds it into one word per workgroup; STORE adds the
// cloud's stores (12 B + 3 B per valid pixel, compacted per workgroup).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mf_probe.hip -o tools/bin/mf_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
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

typedef unsigned int u32x2e __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));

template <int W>
__device__ inline void ldw(const uint8_t* base, uint32_t off, uint32_t soff, uint32_t (&o)[W]) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, 0xffffffff, 0x00020000);
  if constexpr (W == 2) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, 2);
    o[0] = v[0]; o[1] = v[1];
  } else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 2);
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
  }
}

// MODE 0 dense, 1 mf, 2 mf_l2.  W: dwords per lane (2: 8 px, 4: 16 px).
template <int W, int BLOCK, int MODE, int STORE, int TAIL = 0, int LDS_KB = 0, int WAVES = 1>
__global__ __launch_bounds__(BLOCK, WAVES) void probe(const uint8_t* frames, int64_t view_bytes, int tiles_per_view,
                                               const uint8_t* lane_valid, uint32_t* sink, float* xyz, uint8_t* bgr) {
  constexpr int PX = 4 * W;
  constexpr int TILE = BLOCK * PX;
  __shared__ int s_wtot[BLOCK / 64];
  __shared__ uint32_t s_pad[LDS_KB > 0 ? LDS_KB * 256 : 1];   // occupancy: LDS per workgroup
  const int view = blockIdx.x / tiles_per_view, tile = blockIdx.x - view * tiles_per_view;
  const uint8_t* f = frames + view * view_bytes;
  int64_t px0 = int64_t(tile) * TILE + int64_t(threadIdx.x) * PX;
  const bool in = px0 < kNpx;
  if (!in) px0 = 0;
  const uint32_t lp = uint32_t(px0);
  uint32_t w[W], b[W];
  uint32_t valid = 0;
  bool any;
  if constexpr (MODE == 2) {
    any = in && lane_valid[px0 / PX] != 0;
  }
  ldw<W>(f, lp, 0, w);
  ldw<W>(f, lp, uint32_t(kStride), b);
#pragma unroll
  for (int k = 0; k < 4 * W; ++k) {
    const uint32_t wv = (w[k >> 2] >> (8 * (k & 3))) & 0xff, bv = (b[k >> 2] >> (8 * (k & 3))) & 0xff;
    valid |= uint32_t((wv >= 128u) & (wv - bv >= 10u) & in) << k;
  }
  if constexpr (MODE != 2) any = MODE == 0 || valid != 0;
  uint32_t h = 0;
  if (any) {
    uint32_t cp[kNC][W], ci[kNC][W], rp[kNR][W], ri[kNR][W];
#pragma unroll
    for (int g = 0; g < kNC; ++g) {
      ldw<W>(f, lp, uint32_t((2 + 2 * g) * kStride), cp[g]);
      ldw<W>(f, lp, uint32_t((3 + 2 * g) * kStride), ci[g]);
    }
#pragma unroll
    for (int g = 0; g < kNR; ++g) {
      ldw<W>(f, lp, uint32_t((24 + 2 * g) * kStride), rp[g]);
      ldw<W>(f, lp, uint32_t((25 + 2 * g) * kStride), ri[g]);
    }
    uint32_t ac[2 * W] = {}, ar[2 * W] = {};
#pragma unroll
    for (int g = 0; g < kNC; ++g)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const uint32_t m = gt_u8x4(cp[g][k], ci[g][k]);
        ac[2 * k] = (ac[2 * k] << 1) | ((m >> 7) & 0x00010001u);
        ac[2 * k + 1] = (ac[2 * k + 1] << 1) | ((m >> 15) & 0x00010001u);
      }
#pragma unroll
    for (int g = 0; g < kNR; ++g)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const uint32_t m = gt_u8x4(rp[g][k], ri[g][k]);
        ar[2 * k] = (ar[2 * k] << 1) | ((m >> 7) & 0x00010001u);
        ar[2 * k + 1] = (ar[2 * k + 1] << 1) | ((m >> 15) & 0x00010001u);
      }
#pragma unroll
    for (int j = 0; j < 2 * W; ++j) h += gray2bin_x2(ac[j]) * 3u + gray2bin_x2(ar[j]);
  }
  h ^= valid;
  if constexpr (TAIL > 0) {
    // stand-in for phases B-D: TAIL rounds of 4 independent fp64 fma chains (a lane's items)
    double a0 = h, a1 = h + 1, a2 = h + 2, a3 = h + 3;
    for (int i = 0; i < TAIL; ++i) {
      a0 = __builtin_fma(a0, 1.0000001, 0.5); a1 = __builtin_fma(a1, 1.0000001, 0.5);
      a2 = __builtin_fma(a2, 1.0000001, 0.5); a3 = __builtin_fma(a3, 1.0000001, 0.5);
    }
    h += uint32_t(a0 + a1 + a2 + a3);
  }
  if constexpr (LDS_KB > 0) {
    s_pad[threadIdx.x] = h;
    __syncthreads();
    h += s_pad[(threadIdx.x + 64) % BLOCK];
  }
  if constexpr (STORE) {
    // compacted per workgroup: this lane's valid pixels at its block-scan offset
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cnt = __popc(valid);
    int incl = cnt;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_wtot[wave] = incl;
    __syncthreads();
    int off = 0;
    for (int i = 0; i < wave; ++i) off += s_wtot[i];
    const int64_t base = int64_t(blockIdx.x) * TILE + off + incl - cnt;
    int m = 0;
    for (int k = 0; k < PX; ++k)
      if (valid & (1u << k)) {
        const int64_t q = base + m++;
        xyz[3 * q] = float(h); xyz[3 * q + 1] = float(h + k); xyz[3 * q + 2] = float(h + 2);
        bgr[3 * q] = uint8_t(h); bgr[3 * q + 1] = uint8_t(h >> 8); bgr[3 * q + 2] = uint8_t(k);
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

static double g_pattern_bytes[2];   // [W == 4] pattern bytes a view needs at 64-B segments

template <int W, int BLOCK, int MODE, int STORE, int TAIL = 0, int LDS_KB = 0, int WAVES = 1>
void run(const char* name, const uint8_t* frames, int n_views, const uint8_t* lane_valid, uint32_t* sink,
         float* xyz, uint8_t* bgr, int64_t vb) {
  constexpr int TILE = BLOCK * 4 * W;
  const int tpv = int((kNpx + TILE - 1) / TILE);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int it = 0; it < 40; ++it) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((probe<W, BLOCK, MODE, STORE, TAIL, LDS_KB, WAVES>), dim3(tpv * n_views), dim3(BLOCK), 0, 0, frames, vb, tpv,
                       lane_valid, sink, xyz, bgr);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 4) ts.push_back(ms * 1e3f / n_views);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[ts.size() / 2];
  const double need = MODE == 0 ? double(kF) * kNpx : 2.0 * kNpx + g_pattern_bytes[W == 4];
  printf("%-40s %7.2f us/view  frames-needed %6.1f MB  %6.0f GB/s\n", name, us, need / 1e6, need / us / 1e3);
}

int main(int argc, char** argv) {
  const int n_views = 12;
  std::vector<uint8_t> mask(kNpx, 0);
  FILE* fp = fopen(argc > 1 ? argv[1] : "/tmp/mf_mask.bin", "rb");
  if (!fp || fread(mask.data(), 1, kNpx, fp) != size_t(kNpx)) { printf("mask file missing\n"); return 1; }
  fclose(fp);
  for (int wi = 0; wi < 2; ++wi) {
    const int px = wi ? 16 : 8;
    int64_t seg = 0;
    for (int64_t s = 0; s < kNpx / 64; ++s) {
      bool any = false;
      for (int64_t l = 0; l < 64; l += px) {      // a lane reads its whole px span if any is valid
        bool lane = false;
        for (int k = 0; k < px; ++k) lane |= mask[s * 64 + l + k] != 0;
        any |= lane;
      }
      seg += any;
    }
    g_pattern_bytes[wi] = double(seg) * 64 * (kF - 2);
  }
  const int64_t vb = int64_t(kF) * kStride;
  uint8_t* frames; uint32_t* sink;
  CK(hipMalloc(&frames, vb * n_views));
  CK(hipMalloc(&sink, 4096 * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, frames, vb * n_views, 7u);
  std::vector<uint8_t> w(kNpx);
  for (int64_t i = 0; i < kNpx; ++i) w[i] = mask[i] ? 255 : 0;
  for (int v = 0; v < n_views; ++v) {
    CK(hipMemcpy(frames + v * vb, w.data(), kNpx, hipMemcpyHostToDevice));
    CK(hipMemset(frames + v * vb + kStride, 0, kNpx));
  }
  std::vector<uint8_t> lv8(kNpx / 8), lv16(kNpx / 16);
  for (int64_t l = 0; l < kNpx / 8; ++l) for (int k = 0; k < 8; ++k) lv8[l] |= mask[8 * l + k] != 0;
  for (int64_t l = 0; l < kNpx / 16; ++l) for (int k = 0; k < 16; ++k) lv16[l] |= mask[16 * l + k] != 0;
  uint8_t *d_lv8, *d_lv16;
  CK(hipMalloc(&d_lv8, lv8.size() + 4096)); CK(hipMalloc(&d_lv16, lv16.size() + 4096));
  CK(hipMemset(d_lv8, 0, lv8.size() + 4096)); CK(hipMemset(d_lv16, 0, lv16.size() + 4096));
  CK(hipMemcpy(d_lv8, lv8.data(), lv8.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_lv16, lv16.data(), lv16.size(), hipMemcpyHostToDevice));
  float* xyz; uint8_t* bgr;
  CK(hipMalloc(&xyz, int64_t(n_views) * kNpx * 12 + (1 << 20)));
  CK(hipMalloc(&bgr, int64_t(n_views) * kNpx * 3 + (1 << 20)));
  CK(hipDeviceSynchronize());
  int64_t nv = 0;
  for (int64_t i = 0; i < kNpx; ++i) nv += mask[i] != 0;
  printf("mask: %.4f of pixels valid; pattern segments needed %.4f (8 px lanes) %.4f (16 px lanes)\n",
         double(nv) / kNpx, g_pattern_bytes[0] / (42.0 * kNpx), g_pattern_bytes[1] / (42.0 * kNpx));
  const char* only = getenv("MF_PROBE_ONLY");
  if (!only || only[0] != 't') {
    for (int rep = 0; rep < 2; ++rep) {
      run<2, 512, 0, 0>("dense  8px blk512", frames, n_views, d_lv8, sink, xyz, bgr, vb);
      run<2, 512, 1, 0>("mf     8px blk512", frames, n_views, d_lv8, sink, xyz, bgr, vb);
      run<2, 512, 2, 0>("mf_l2  8px blk512", frames, n_views, d_lv8, sink, xyz, bgr, vb);
      run<4, 256, 1, 0>("mf16  16px blk256", frames, n_views, d_lv16, sink, xyz, bgr, vb);
      run<4, 256, 2, 0>("mf16_l2 16px blk256", frames, n_views, d_lv16, sink, xyz, bgr, vb);
      run<2, 512, 1, 1>("mf     8px blk512 + stores", frames, n_views, d_lv8, sink, xyz, bgr, vb);
      run<2, 512, 2, 1>("mf_l2  8px blk512 + stores", frames, n_views, d_lv8, sink, xyz, bgr, vb);
      run<2, 512, 0, 1>("dense  8px blk512 + stores", frames, n_views, d_lv8, sink, xyz, bgr, vb);
    }
  }
  // occupancy vs a compute tail: 2 workgroups per CU (70 KB LDS each) against 3 (50 KB), a
  // tail of 0 / 150 / 300 rounds of 4 fp64 fma chains (~ phases B-D of main3: 600-1200 VALU)
  for (int rep = 0; rep < 2; ++rep) {
    run<2, 512, 1, 0, 0, 70, 4>("mf tail0   2 WG/CU", frames, n_views, d_lv8, sink, xyz, bgr, vb);
    run<2, 512, 1, 0, 0, 50, 6>("mf tail0   3 WG/CU", frames, n_views, d_lv8, sink, xyz, bgr, vb);
    run<2, 512, 1, 0, 150, 70, 4>("mf tail150 2 WG/CU", frames, n_views, d_lv8, sink, xyz, bgr, vb);
    run<2, 512, 1, 0, 150, 50, 6>("mf tail150 3 WG/CU", frames, n_views, d_lv8, sink, xyz, bgr, vb);
    run<2, 512, 1, 0, 300, 70, 4>("mf tail300 2 WG/CU", frames, n_views, d_lv8, sink, xyz, bgr, vb);
    run<2, 512, 1, 0, 300, 50, 6>("mf tail300 3 WG/CU", frames, n_views, d_lv8, sink, xyz, bgr, vb);
    run<2, 512, 1, 0, 300, 35, 8>("mf tail300 4 WG/CU", frames, n_views, d_lv8, sink, xyz, bgr, vb);
  }
  return 0;
}
