// fetch_probe.hip -- calibration microbenchmark (not product code): what rocprofv3's HBM byte
// counters report for main3's access shapes, against byte counts known exactly on the host
// (VERDICT r3 weak #3 / next #2).
//
// Read variants (one lane = 8 or 16 consecutive pixels of each of NF pattern frames, frame f at
// byte f * stride, stride % 256 == 0, the buffer_load_b64/b128 + aux 2 main3 uses):
//   dense16  every lane reads 16 B of every frame            (the guide's calibrated shape)
//   dense8   every lane reads 8 B of every frame             (main3's load width, no mask)
//   mf8      8 B per frame only in lanes whose mask byte is set (main3's mask-first shape); the
//            lane decision comes from a 1-byte-per-lane table (its bytes reported separately)
//   mf16     16 B per frame in lanes of 16 pixels holding a valid one: the same 128-B lines as
//            mf8 (a lane's 16 bytes never straddle one), half the load instructions
// Write variants (lane i writes record i, consecutive lanes consecutive records):
//   st16     16 B per lane (dwordx4, the guide's calibrated shape)
//   st12     12 B per lane (dwordx3: main3's XYZ stores)
//   st3      3 B per lane (short + byte: main3's BGR stores)
// Every variant runs over NCOPY buffer copies (> 256 MiB in total, so nothing stays in the
// Infinity Cache between dispatches), one dispatch per copy, REPS rounds.
// The host prints one JSON line: per variant the exact bytes requested per dispatch, and for the
// read variants the bytes of the 32-, 64- and 128-byte aligned blocks that hold a requested byte.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/fetch_probe.hip -o <bin>
//   <bin> [mask.bin]      mask.bin: one byte per pixel of a 1920x1080 view (nonzero = valid)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <set>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kNF = 42, kNCOPY = 4, kREPS = 2, kBlock = 256;
constexpr int64_t kW = 1920, kH = 1080, kNpx = kW * kH, kStride = (kNpx + 255) / 256 * 256;

template <int PX, int MF>
__global__ __launch_bounds__(kBlock) void rd_kernel(const uint8_t* frames, const uint8_t* lane_valid, int64_t n_lanes,
                                                    uint32_t* sink) {
  const int64_t lane = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (lane >= n_lanes) return;
  if (MF && !lane_valid[lane]) return;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(frames), 0, 0xffffffff, 0x00020000);
  const uint32_t off = uint32_t(lane * PX);
  uint32_t acc = 0;
#pragma unroll
  for (int f = 0; f < kNF; ++f) {
    if constexpr (PX == 16) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, uint32_t(f * kStride), 2);
      acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    } else {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, uint32_t(f * kStride), 2);
      acc ^= v[0] ^ v[1];
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;          // keeps the loads; (practically) never stores
}

template <int BYTES>
__global__ __launch_bounds__(kBlock) void st_kernel(uint8_t* out, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = uint32_t(i) * 2654435761u;
  if constexpr (BYTES == 16) {
    reinterpret_cast<uint4*>(out)[i] = make_uint4(v, v + 1, v + 2, v + 3);
  } else if constexpr (BYTES == 12) {
    float* o = reinterpret_cast<float*>(out) + 3 * i;
    o[0] = float(v); o[1] = float(v + 1); o[2] = float(v + 2);
  } else {
    uint8_t* o = out + 3 * i;
    o[0] = uint8_t(v); o[1] = uint8_t(v >> 8); o[2] = uint8_t(v >> 16);
  }
}

static int64_t blocks_holding(const std::vector<uint8_t>& lv, int px, int block) {
  // distinct aligned `block`-byte blocks holding a requested byte, over all NF frames
  int64_t n = 0;
  for (int f = 0; f < kNF; ++f) {
    int64_t last = -1;
    for (size_t l = 0; l < lv.size(); ++l) {
      if (!lv[l]) continue;
      const int64_t b0 = (f * kStride + int64_t(l) * px) / block, b1 = (f * kStride + int64_t(l) * px + px - 1) / block;
      for (int64_t b = b0; b <= b1; ++b)
        if (b != last) { ++n; last = b; }
    }
  }
  return n;
}

int main(int argc, char** argv) {
  const int64_t lanes8 = kNpx / 8, lanes16 = kNpx / 16;
  std::vector<uint8_t> mask(kNpx, 1);
  if (argc > 1) {
    FILE* fp = fopen(argv[1], "rb");
    if (!fp || fread(mask.data(), 1, kNpx, fp) != size_t(kNpx)) { printf("bad mask file\n"); return 1; }
    fclose(fp);
  }
  std::vector<uint8_t> lv(lanes8, 0), lv16(lanes16, 0), all8(lanes8, 1), all16(lanes16, 1);
  int64_t valid_lanes = 0, valid_px = 0, valid_lanes16 = 0;
  for (int64_t l = 0; l < lanes8; ++l) {
    for (int k = 0; k < 8; ++k) lv[l] |= mask[8 * l + k] != 0, valid_px += mask[8 * l + k] != 0;
    valid_lanes += lv[l];
  }
  for (int64_t l = 0; l < lanes16; ++l) {
    lv16[l] = lv[2 * l] | lv[2 * l + 1];
    valid_lanes16 += lv16[l];
  }
  const size_t view = size_t(kNF) * kStride;
  std::vector<uint8_t*> bufs(kNCOPY);
  std::vector<uint8_t> host(view);
  for (size_t i = 0; i < view; ++i) host[i] = uint8_t(i * 131 + (i >> 11));
  for (auto& b : bufs) { CK(hipMalloc(&b, view)); CK(hipMemcpy(b, host.data(), view, hipMemcpyHostToDevice)); }
  uint8_t* d_lv; uint32_t* sink;
  CK(hipMalloc(&d_lv, lanes8)); CK(hipMemcpy(d_lv, lv.data(), lanes8, hipMemcpyHostToDevice));
  uint8_t* d_lv16;
  CK(hipMalloc(&d_lv16, lanes16)); CK(hipMemcpy(d_lv16, lv16.data(), lanes16, hipMemcpyHostToDevice));
  CK(hipMalloc(&sink, 64));
  const int64_t n_st = 4 << 20;                    // records per store dispatch
  std::vector<uint8_t*> obufs(kNCOPY);
  for (auto& b : obufs) CK(hipMalloc(&b, n_st * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    launch(0);                                      // warm (not in the REPS x NCOPY count below)
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < kREPS; ++r)
      for (int c = 0; c < kNCOPY; ++c) launch(c);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3 * ms / (kREPS * kNCOPY);
  };
  const unsigned g8 = unsigned((lanes8 + kBlock - 1) / kBlock), g16 = unsigned((lanes16 + kBlock - 1) / kBlock);
  const double t_d16 = timeit([&](int c) { hipLaunchKernelGGL((rd_kernel<16, 0>), dim3(g16), dim3(kBlock), 0, 0, bufs[c], nullptr, lanes16, sink); });
  const double t_d8 = timeit([&](int c) { hipLaunchKernelGGL((rd_kernel<8, 0>), dim3(g8), dim3(kBlock), 0, 0, bufs[c], nullptr, lanes8, sink); });
  const double t_mf = timeit([&](int c) { hipLaunchKernelGGL((rd_kernel<8, 1>), dim3(g8), dim3(kBlock), 0, 0, bufs[c], d_lv, lanes8, sink); });
  const double t_mf16 = timeit([&](int c) { hipLaunchKernelGGL((rd_kernel<16, 1>), dim3(g16), dim3(kBlock), 0, 0, bufs[c], d_lv16, lanes16, sink); });
  const unsigned gs = unsigned((n_st + kBlock - 1) / kBlock);
  const double t_s16 = timeit([&](int c) { hipLaunchKernelGGL(st_kernel<16>, dim3(gs), dim3(kBlock), 0, 0, obufs[c], n_st); });
  const double t_s12 = timeit([&](int c) { hipLaunchKernelGGL(st_kernel<12>, dim3(gs), dim3(kBlock), 0, 0, obufs[c], n_st); });
  const double t_s3 = timeit([&](int c) { hipLaunchKernelGGL(st_kernel<3>, dim3(gs), dim3(kBlock), 0, 0, obufs[c], n_st); });
  CK(hipDeviceSynchronize());
  const int64_t req_dense = int64_t(kNF) * kNpx, req_mf = int64_t(kNF) * 8 * valid_lanes;
  printf("{\"frames\": %d, \"stride\": %lld, \"copies\": %d, \"reps\": %d, \"dispatches_per_variant\": %d, "
         "\"valid_px\": %lld, \"valid_lanes8\": %lld, \"lanes8\": %lld, \"lane_table_bytes\": %lld, \"variants\": {",
         kNF, (long long)kStride, kNCOPY, kREPS, 1 + kREPS * kNCOPY, (long long)valid_px, (long long)valid_lanes,
         (long long)lanes8, (long long)lanes8);
  printf("\"rd_kernel<16, 0>\": {\"what\": \"dense16\", \"requested\": %lld, \"b32\": %lld, \"b64\": %lld, \"b128\": %lld, \"us\": %.2f}, ",
         (long long)req_dense, (long long)blocks_holding(all16, 16, 32) * 32, (long long)blocks_holding(all16, 16, 64) * 64,
         (long long)blocks_holding(all16, 16, 128) * 128, t_d16);
  printf("\"rd_kernel<8, 0>\": {\"what\": \"dense8\", \"requested\": %lld, \"b32\": %lld, \"b64\": %lld, \"b128\": %lld, \"us\": %.2f}, ",
         (long long)req_dense, (long long)blocks_holding(all8, 8, 32) * 32, (long long)blocks_holding(all8, 8, 64) * 64,
         (long long)blocks_holding(all8, 8, 128) * 128, t_d8);
  printf("\"rd_kernel<8, 1>\": {\"what\": \"mf8\", \"requested\": %lld, \"b32\": %lld, \"b64\": %lld, \"b128\": %lld, \"us\": %.2f}, ",
         (long long)req_mf, (long long)blocks_holding(lv, 8, 32) * 32, (long long)blocks_holding(lv, 8, 64) * 64,
         (long long)blocks_holding(lv, 8, 128) * 128, t_mf);
  printf("\"rd_kernel<16, 1>\": {\"what\": \"mf16\", \"requested\": %lld, \"b32\": %lld, \"b64\": %lld, \"b128\": %lld, \"us\": %.2f}, ",
         (long long)(int64_t(kNF) * 16 * valid_lanes16), (long long)blocks_holding(lv16, 16, 32) * 32,
         (long long)blocks_holding(lv16, 16, 64) * 64, (long long)blocks_holding(lv16, 16, 128) * 128, t_mf16);
  printf("\"st_kernel<16>\": {\"what\": \"st16\", \"requested\": %lld, \"us\": %.2f}, ", (long long)(16 * n_st), t_s16);
  printf("\"st_kernel<12>\": {\"what\": \"st12\", \"requested\": %lld, \"us\": %.2f}, ", (long long)(12 * n_st), t_s12);
  printf("\"st_kernel<3>\": {\"what\": \"st3\", \"requested\": %lld, \"us\": %.2f}}}\n", (long long)(3 * n_st), t_s3);
  return 0;
}
