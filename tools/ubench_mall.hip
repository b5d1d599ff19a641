// Microbenchmark: does a write of S bytes read back right away cost HBM bandwidth, or is the
// round trip served by the 256 MB Infinity Cache (MALL)? Prices a chunked stage -> transpose
// for kernel 9 (G_A written and read back per chunk instead of 4 GB written, then read).
//   * ring1:  write S, read S, always the same S bytes (dirty lines rewritten while cached)
//   * cycle:  write S, read the same S, next pair at the next S bytes of an 8 GB region
//   * far:    write S at one offset, read S at another (no reuse: the HBM round trip)
//   * reread: read the same S again and again
// GB/s = bytes moved by the kernels (2 S per pair) / device time.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_mall.hip -o tools/bin/ubench_mall
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

__global__ __launch_bounds__(256) void k_write(float4 *__restrict__ dst, long long n4, float v) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride)
    dst[i] = make_float4(v, v + 1.f, v + 2.f, (float)(i & 7));
}

__global__ __launch_bounds__(256) void k_read(const float4 *__restrict__ src, long long n4, float *__restrict__ out) {
  const long long stride = (long long)gridDim.x * 256;
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    const float4 x = src[i];
    acc += x.x + x.y + x.z + x.w;
  }
  if (acc == -1.2345f) out[blockIdx.x] = acc;  // never true: keeps the loads
}

int main() {
  const long long REGION = 8LL << 30;
  char *base;
  float *out;
  CK(hipMalloc(&base, REGION));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(base, 0, REGION));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 8;
  const long long sizes_mb[] = {16, 32, 64, 96, 128, 192, 256, 512};
  printf("%8s %10s %10s %10s %10s\n", "S_MB", "ring1", "cycle", "far", "reread");
  for (long long smb : sizes_mb) {
    const long long S = smb << 20, n4 = S / 16;
    const int pairs = (int)((96LL << 30) / (2 * S));  // ~96 GB moved per mode
    const long long slots = REGION / S;
    double gbs[4];
    for (int mode = 0; mode < 4; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int k = 0; k < pairs; ++k) {
          char *w, *r;
          if (mode == 0) {
            w = r = base;
          } else if (mode == 1) {
            w = r = base + (k % slots) * S;
          } else if (mode == 2) {
            w = base + ((2 * k) % slots) * S;
            r = base + ((2 * k + slots / 2 + 1) % slots) * S;
          } else {
            w = nullptr;
            r = base;
          }
          if (w) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (float4 *)w, n4, (float)k);
          hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const float4 *)r, n4, out);
          if (!w) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const float4 *)r, n4, out);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        gbs[mode] = 2.0 * S * pairs / (ms * 1e-3) / 1e9;
      }
    }
    printf("%8lld %10.0f %10.0f %10.0f %10.0f\n", smb, gbs[0], gbs[1], gbs[2], gbs[3]);
    fflush(stdout);
  }
  CK(hipGetLastError());
  return 0;
}
