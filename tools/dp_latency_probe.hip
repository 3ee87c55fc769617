// dp_latency_probe.hip -- clocks per dependent fp64 op on gfx950 (s_memtime around a chain of
// 1024 dependent v_add_f64 / v_fma_f64), with the whole wave active and with one lane active:
// the cost model of otsu_wave's serial chains (tools/otsu_probe.hip).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off tools/dp_latency_probe.hip -o tools/bin/dp_latency_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(64) void chain(const double* in, double* out, uint64_t* clk) {
  const int lane = threadIdx.x;
  double x = in[lane], y = in[64 + lane], z = in[128 + lane];
  uint64_t c0 = 0, c1 = 0;
  __builtin_amdgcn_s_waitcnt(0);
  c0 = __builtin_amdgcn_s_memtime();
  if (MODE < 2 || lane == 0) {
#pragma unroll 64
    for (int i = 0; i < 1024; ++i) {
      if (MODE == 0 || MODE == 2) x = x + y;
      else x = __builtin_fma(x, y, z);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  out[lane] = x;
  __builtin_amdgcn_s_waitcnt(0);
  c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) clk[MODE] = c1 - c0;
}

int main() {
  double h[192];
  for (int i = 0; i < 192; ++i) h[i] = 1.0 + i * 1e-9;
  double *din, *dout;
  uint64_t* dclk;
  hipMalloc(&din, sizeof(h));
  hipMalloc(&dout, 64 * 8);
  hipMalloc(&dclk, 8 * 8);
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, din, dout, dclk);
    hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, din, dout, dclk);
    hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, din, dout, dclk);
    hipLaunchKernelGGL(chain<3>, dim3(1), dim3(64), 0, 0, din, dout, dclk);
  }
  uint64_t c[8];
  hipMemcpy(c, dclk, sizeof(c), hipMemcpyDeviceToHost);
  printf("{\"add_wave\": %.1f, \"fma_wave\": %.1f, \"add_lane0\": %.1f, \"fma_lane0\": %.1f, \"unit\": \"clocks per dependent op\"}\n",
         c[0] / 1024.0, c[1] / 1024.0, c[2] / 1024.0, c[3] / 1024.0);
  return 0;
}
