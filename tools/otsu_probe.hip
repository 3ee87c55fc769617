// otsu_probe.hip -- times the Otsu tail (otsu_wave of csrc/slgpu.hip, OpenCV's sequential fp64
// chains) on one wave, alone on the GPU, with s_memrealtime (100 MHz) around each part, and
// checks its threshold against the host restatement below (the same loop as the oracle's
// otsu_from_hist, oracle/sl_oracle.py).  Histograms: argv[1] = a file of uint32 [k][256] (e.g.
// tools/otsu_probe.py writes a C2 view's white and clip(white - black) histograms), else
// synthetic bimodal ones.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off tools/otsu_probe.hip -o /tmp/otsu_probe
__device__ unsigned long long g_otsu_marks[8];
#define SLG_OTSU_MARK(k) (__builtin_amdgcn_s_waitcnt(0), g_otsu_marks[k] = __builtin_amdgcn_s_memtime())
#include "../structured_light_for_3d_model_replication_amd/csrc/slgpu.hip"


#include <float.h>
#include <algorithm>
#include <vector>

namespace {

__global__ __launch_bounds__(64) void otsu_probe_kernel(const uint32_t* hists, int64_t n, int reps, double* thr,
                                                        uint64_t* ticks) {
  __shared__ uint32_t h[256];
  __shared__ __attribute__((aligned(16))) double lds[kOtsuLds];
  const int k = blockIdx.x;
  for (int i = threadIdx.x; i < 256; i += 64) h[i] = hists[k * 256 + i];
  __syncthreads();
  double t = 0.0;
  uint64_t best = ~0ull, best_clk = ~0ull;
  for (int r = 0; r < reps; ++r) {
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    t = otsu_wave(h, n, lds);
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (t1 - t0 < best) { best = t1 - t0; best_clk = c1 - c0; }
    n += (t == -1.0);                      // (keeps the calls from being merged)
  }
  if (threadIdx.x == 0) {
    thr[k] = t;
    ticks[2 * k] = best;
    ticks[2 * k + 1] = best_clk;
  }
}

// OpenCV getThreshVal_Otsu_8u, sequential (the oracle's restatement)
double otsu_host(const uint32_t* h, int64_t n) {
  const double scale = 1.0 / double(n);
  double mu = 0.0;
  for (int i = 0; i < 256; ++i) mu += double(i) * double(h[i]);
  mu *= scale;
  double mu1 = 0.0, q1 = 0.0, max_sigma = 0.0, max_val = 0.0;
  for (int i = 0; i < 256; ++i) {
    const double p_i = double(h[i]) * scale;
    mu1 *= q1;
    q1 += p_i;
    const double q2 = 1.0 - q1;
    if (std::min(q1, q2) < double(FLT_EPSILON) || std::max(q1, q2) > 1.0 - double(FLT_EPSILON)) continue;
    mu1 = (mu1 + double(i) * p_i) / q1;
    const double mu2 = (mu - q1 * mu1) / q2;
    const double sigma = q1 * q2 * (mu1 - mu2) * (mu1 - mu2);
    if (sigma > max_sigma) { max_sigma = sigma; max_val = double(i); }
  }
  return max_val;
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<uint32_t> hs;
  if (argc > 1) {
    FILE* f = fopen(argv[1], "rb");
    if (!f) { printf("cannot open %s\n", argv[1]); return 2; }
    uint32_t v;
    while (fread(&v, 4, 1, f) == 1) hs.push_back(v);
    fclose(f);
  } else {
    hs.assign(2 * 256, 0);
    for (int i = 0; i < 256; ++i) {
      hs[i] = uint32_t(2000.0 * exp(-0.5 * ((i - 30) / 8.0) * ((i - 30) / 8.0)) + 9000.0 * exp(-0.5 * ((i - 190) / 12.0) * ((i - 190) / 12.0)));
      hs[256 + i] = uint32_t(5000.0 * exp(-0.5 * ((i - 5) / 3.0) * ((i - 5) / 3.0)) + 7000.0 * exp(-0.5 * ((i - 170) / 10.0) * ((i - 170) / 10.0)));
    }
  }
  const int k = int(hs.size() / 256);
  int rc = 0;
  uint32_t *dh;
  double* dthr;
  uint64_t* dt;
  hipMalloc(&dh, hs.size() * 4);
  hipMalloc(&dthr, k * 8);
  hipMalloc(&dt, 2 * k * 8);
  hipMemcpy(dh, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
  for (int j = 0; j < k; ++j) {
    int64_t n = 0;
    for (int i = 0; i < 256; ++i) n += hs[j * 256 + i];
    hipLaunchKernelGGL(otsu_probe_kernel, dim3(1), dim3(64), 0, 0, dh + j * 256, n, 20, dthr, dt);
    double thr = 0;
    unsigned long long marks[8];
    hipMemcpyFromSymbol(marks, HIP_SYMBOL(g_otsu_marks), sizeof(marks));
    printf("{\"hist\": %d, \"part_clocks\": [", j);
    for (int q = 1; q < 8; ++q) printf("%llu%s", marks[q] - marks[q - 1], q < 7 ? ", " : "]}\n");
    uint64_t ticks[2] = {0, 0};
    hipMemcpy(&thr, dthr, 8, hipMemcpyDeviceToHost);
    hipMemcpy(ticks, dt, 16, hipMemcpyDeviceToHost);
    const double want = otsu_host(&hs[j * 256], n);
    printf("{\"hist\": %d, \"n\": %lld, \"thr\": %.1f, \"host\": %.1f, \"us\": %.2f, \"clocks\": %llu, "
           "\"clocks_per_bin\": %.1f}\n", j, (long long)n, thr, want, ticks[0] / 100.0,
           (unsigned long long)ticks[1], ticks[1] / 256.0);
    if (thr != want) rc = 1;
  }
  return rc;
}
