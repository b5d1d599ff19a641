// PMC calibration for the round kernel's access widths (MI355X_MICROARCH.md § HBM: only
// 16-B-per-lane streams are calibrated there). Each kernel moves a KNOWN byte count through
// HBM with one access width, on buffers far larger than the 256 MiB Infinity Cache:
//   k_read8  : 8 B per lane loads (fp64 flows / node arrays), 512 MiB
//   k_read4  : 4 B per lane loads (col, rowptr), 512 MiB
//   k_write8 : 8 B per lane stores, 512 MiB
// tools/pmc_summary.py divides each counter by these byte counts and corrects the round
// kernel's FETCH_SIZE / WRITE_SIZE with the 8-B factors (most of its bytes are 8-B streams).
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/bin/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      exit(1);                                                      \
    }                                                               \
  } while (0)

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T *__restrict__ p, long long n, double *__restrict__ out) {
  double acc = 0.0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    acc += (double)p[i];
  if (acc == 1.2345) out[0] = acc;  // keep the loads live, store ~never
}

__global__ __launch_bounds__(256) void k_write8(double *__restrict__ p, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = (double)i;
}

int main() {
  const size_t bytes = 512ull << 20;
  void *buf = nullptr;
  double *out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(buf, 0, bytes));
  const int grid = 256 * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](const char *name, auto launch) {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"kernel\": \"%s\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", name, bytes, ms, bytes / (ms * 1e6));
  };
  timed("calib_read8", [&] { hipLaunchKernelGGL(k_read<double>, dim3(grid), dim3(256), 0, 0, (const double *)buf, (long long)(bytes / 8), out); });
  timed("calib_read4", [&] { hipLaunchKernelGGL(k_read<int>, dim3(grid), dim3(256), 0, 0, (const int *)buf, (long long)(bytes / 4), out); });
  timed("calib_write8", [&] { hipLaunchKernelGGL(k_write8, dim3(grid), dim3(256), 0, 0, (double *)buf, (long long)(bytes / 8)); });
  CK(hipDeviceSynchronize());
  return 0;
}
