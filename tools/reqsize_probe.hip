// reqsize_probe.hip -- calibration microbenchmark (not product code): does any gfx950 cache
// policy make main3's mask-gated 8-byte pattern loads fetch 64-byte HBM requests instead of
// 128-byte lines?  (round 4: rocprofv3 shows ~100 % TCC_EA0_RDREQ_128B for main3, while the
// 64-byte segments holding a valid pixel are 20 % fewer bytes than the 128-byte lines.)
// One kernel per buffer-load cache-policy immediate (gfx940+: 1 sc0, 2 nt, 16 sc1), same mask-
// gated shape as fetch_probe.hip's mf8 (lane = 8 px of each of 42 frames, only lanes with a
// valid pixel load).  Prints one JSON line: per policy the mean dispatch time; the request
// sizes come from a separate rocprofv3 --pmc pass over the same binary (kernel names carry AUX).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/reqsize_probe.hip -o <bin>;  <bin> mask.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kNF = 42, kNCOPY = 4, kREPS = 2, kBlock = 256;
constexpr int64_t kW = 1920, kH = 1080, kNpx = kW * kH, kStride = (kNpx + 255) / 256 * 256;

template <int AUX>
__global__ __launch_bounds__(kBlock) void mf8_policy(const uint8_t* frames, const uint8_t* lane_valid, int64_t n_lanes,
                                                     uint32_t* sink) {
  const int64_t lane = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (lane >= n_lanes || !lane_valid[lane]) return;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(frames), 0, 0xffffffff, 0x00020000);
  const uint32_t off = uint32_t(lane * 8);
  uint32_t acc = 0;
#pragma unroll
  for (int f = 0; f < kNF; ++f) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, uint32_t(f * kStride), AUX);
    acc ^= v[0] ^ v[1];
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;          // keeps the loads; (practically) never stores
}

int main(int argc, char** argv) {
  const int64_t lanes8 = kNpx / 8;
  std::vector<uint8_t> mask(kNpx, 1);
  if (argc > 1) {
    FILE* fp = fopen(argv[1], "rb");
    if (!fp || fread(mask.data(), 1, kNpx, fp) != size_t(kNpx)) { printf("bad mask file\n"); return 1; }
    fclose(fp);
  }
  std::vector<uint8_t> lv(lanes8, 0);
  int64_t valid_lanes = 0;
  for (int64_t l = 0; l < lanes8; ++l) {
    for (int k = 0; k < 8; ++k) lv[l] |= mask[8 * l + k] != 0;
    valid_lanes += lv[l];
  }
  const size_t view = size_t(kNF) * kStride;
  std::vector<uint8_t*> bufs(kNCOPY);
  std::vector<uint8_t> host(view);
  for (size_t i = 0; i < view; ++i) host[i] = uint8_t(i * 131 + (i >> 11));
  for (auto& b : bufs) { CK(hipMalloc(&b, view)); CK(hipMemcpy(b, host.data(), view, hipMemcpyHostToDevice)); }
  uint8_t* d_lv; uint32_t* sink;
  CK(hipMalloc(&d_lv, lanes8)); CK(hipMemcpy(d_lv, lv.data(), lanes8, hipMemcpyHostToDevice));
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const unsigned g8 = unsigned((lanes8 + kBlock - 1) / kBlock);
  auto timeit = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(g8), dim3(kBlock), 0, 0, bufs[0], d_lv, lanes8, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < kREPS; ++r)
      for (int c = 0; c < kNCOPY; ++c) hipLaunchKernelGGL(kern, dim3(g8), dim3(kBlock), 0, 0, bufs[c], d_lv, lanes8, sink);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3 * ms / (kREPS * kNCOPY);
  };
  printf("{\"valid_lanes8\": %lld, \"lanes8\": %lld, \"requested_per_dispatch\": %lld, \"us\": {", (long long)valid_lanes,
         (long long)lanes8, (long long)(int64_t(kNF) * 8 * valid_lanes));
  printf("\"0\": %.2f, ", timeit(mf8_policy<0>));
  printf("\"1\": %.2f, ", timeit(mf8_policy<1>));
  printf("\"2\": %.2f, ", timeit(mf8_policy<2>));
  printf("\"3\": %.2f, ", timeit(mf8_policy<3>));
  printf("\"16\": %.2f, ", timeit(mf8_policy<16>));
  printf("\"17\": %.2f, ", timeit(mf8_policy<17>));
  printf("\"18\": %.2f, ", timeit(mf8_policy<18>));
  printf("\"19\": %.2f}}\n", timeit(mf8_policy<19>));
  return 0;
}
