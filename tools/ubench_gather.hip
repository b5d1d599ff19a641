// Microbenchmark: random fp64 gathers from a table of T bytes (8M gathers, indices streamed
// coalesced) vs a pure coalesced stream of the same index+value bytes. Prices the
// a_{r-1}[col e] gather of the round kernel on MI355X.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_gather.hip -o /tmp/ubench_gather
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s: %s\n", #x, hipGetErrorString(e));                            \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int PER>
__global__ __launch_bounds__(256) void k_gather(const int *__restrict__ idx, const double *__restrict__ tab,
                                                double *__restrict__ out, int n) {
  int base = (blockIdx.x * 256) * PER + threadIdx.x;
  double acc = 0.0;
  int c[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) c[k] = base + k * 256 < n ? idx[base + k * 256] : 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) acc += tab[c[k]];
  if (acc == 1.2345) out[0] = acc;
}

template <int PER>
__global__ __launch_bounds__(256) void k_gather_store(const int *__restrict__ idx, const double *__restrict__ tab,
                                                      double *__restrict__ out, int n) {
  int base = (blockIdx.x * 256) * PER + threadIdx.x;
  int c[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) c[k] = base + k * 256 < n ? idx[base + k * 256] : 0;
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (base + k * 256 < n) out[base + k * 256] = tab[c[k]];
}

__global__ void k_stream(const int *__restrict__ idx, const double *__restrict__ src, double *__restrict__ out,
                         int n) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = src[i] + (double)idx[i];
}

int main() {
  const int n = 8 * 1000 * 1000;
  std::vector<int> h(n);
  int *d_idx;
  double *d_tab, *d_out, *d_src;
  CK(hipMalloc(&d_idx, sizeof(int) * n));
  CK(hipMalloc(&d_out, sizeof(double) * n));
  CK(hipMalloc(&d_src, sizeof(double) * n));
  CK(hipMalloc(&d_tab, sizeof(double) * (64 << 20)));
  CK(hipMemset(d_tab, 0, sizeof(double) * (64 << 20)));
  CK(hipMemset(d_src, 0, sizeof(double) * n));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  unsigned long long s = 88172645463325252ull;
  for (long long tb : {1ll << 20, 2ll << 20, 4ll << 20, 8ll << 20, 16ll << 20, 64ll << 20, 256ll << 20}) {
    long long entries = tb / 8;
    for (int i = 0; i < n; ++i) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      h[i] = (int)(s % (unsigned long long)entries);
    }
    CK(hipMemcpy(d_idx, h.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    for (int variant = 0; variant < 2; ++variant) {
      float best = 1e9;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a));
        for (int it = 0; it < 20; ++it) {
          if (variant == 0)
            hipLaunchKernelGGL(k_gather<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, d_idx, d_tab, d_out, n);
          else
            hipLaunchKernelGGL(k_gather_store<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, d_idx, d_tab, d_out, n);
        }
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      double us = best / 20 * 1e3;
      printf("table %6lld KB  %-13s %8.1f us  %6.1f Ggathers/s\n", tb >> 10,
             variant == 0 ? "gather" : "gather+store", us, n / us / 1e3);
    }
  }
  float best = 1e9;
  for (int rep = 0; rep < 6; ++rep) {
    CK(hipEventRecord(a));
    for (int it = 0; it < 20; ++it)
      hipLaunchKernelGGL(k_stream, dim3((n + 255) / 256), dim3(256), 0, 0, d_idx, d_src, d_out, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  double us = best / 20 * 1e3;
  printf("stream 20B/elem x 8M: %8.1f us  %6.0f GB/s\n", us, 20.0 * n / us / 1e3);
  return 0;
}
