// mfma_hist_probe.hip -- checks (and times) the 256-bin byte histogram on the i8 matrix cores
// used by stats_kernel: for 64 pixels v_k, A[m][k] = [v_k >> 4 == m], B[k][n] = [v_k & 15 == n],
// so one v_mfma_i32_16x16x64_i8 adds hist[16m + n].  Verifies the A/B lane maps against a CPU
// count on skewed random data (exit code 1 on any mismatch).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mfma_hist_probe.hip -o /tmp/mfma_hist_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ inline uint32_t eq_nib(uint32_t x, uint32_t rep) {   // bytes (< 16) equal -> 0x01
  const uint32_t t = x ^ rep;
  return (~((t | 0x80808080u) - 0x01010101u) >> 7) & 0x01010101u;
}

__global__ void hist_mfma(const uint8_t* data, int64_t n, uint32_t* hist) {
  const int lane = threadIdx.x & 63;
  const int sel = lane & 15;
  const uint32_t rep = uint32_t(sel) * 0x01010101u;
  v4i acc = {0, 0, 0, 0};
  for (int64_t c = (int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6)) * 1024; c < n;
       c += int64_t(gridDim.x) * (blockDim.x / 64) * 1024) {
    uint32_t d[4];
    const int64_t o = c + 16 * lane;
    for (int q = 0; q < 4; ++q) {
      uint32_t w = 0;
      for (int b = 0; b < 4; ++b)
        if (o + 4 * q + b < n) w |= uint32_t(data[o + 4 * q + b]) << (8 * b);
      d[q] = w;
    }
    for (int i = 0; i < 16; ++i) {
      const int src = 4 * i + (lane >> 4);
      v4i a, b;
      for (int q = 0; q < 4; ++q) {
        const uint32_t x = uint32_t(__shfl(int(d[q]), src));
        // validity: pixel c + 16*src + 4q + byte < n
        uint32_t vmask = 0;
        for (int bb = 0; bb < 4; ++bb) vmask |= (c + 16 * src + 4 * q + bb < n ? 0x01u : 0u) << (8 * bb);
        a[q] = int(eq_nib((x >> 4) & 0x0f0f0f0fu, rep) & vmask);
        b[q] = int(eq_nib(x & 0x0f0f0f0fu, rep));
      }
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc, 0, 0, 0);
    }
  }
  // C/D: col = lane & 15, row = (lane >> 4) * 4 + r
  for (int r = 0; r < 4; ++r) {
    const int row = (lane >> 4) * 4 + r, col = lane & 15;
    if (acc[r]) atomicAdd(&hist[16 * row + col], uint32_t(acc[r]));
  }
}

int main() {
  const int64_t n = 2073600 + 77;
  std::vector<uint8_t> h(n);
  uint64_t s = 12345;
  for (int64_t i = 0; i < n; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t r = uint32_t(s >> 33);
    h[i] = (r % 3 == 0) ? uint8_t(10 + (r >> 8) % 8) : uint8_t(r >> 13);   // skew + uniform
  }
  std::vector<uint32_t> ref(256, 0);
  for (int64_t i = 0; i < n; ++i) ref[h[i]]++;
  uint8_t* dd; uint32_t* dh;
  hipMalloc(&dd, n + 64); hipMalloc(&dh, 1024);
  hipMemcpy(dd, h.data(), n, hipMemcpyHostToDevice);
  hipMemset(dh, 0, 1024);
  hipLaunchKernelGGL(hist_mfma, dim3(128), dim3(256), 0, 0, dd, n, dh);
  std::vector<uint32_t> got(256);
  hipMemcpy(got.data(), dh, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += got[i] != ref[i];
  printf("bins mismatching: %d (bin 12: got %u want %u)\n", bad, got[12], ref[12]);
  return bad != 0;
}
