// Microbenchmark: the streaming ceiling of the part, to price what "at the copy rate" means
// for the round kernels (ER-1M rounds move their traffic at 5.0-5.4 TB/s; bench.py's
// fu_copy_bandwidth float4 copy measures 5.1-5.5 TB/s on the boxes; MI355X_MICROARCH.md
// quotes 6.29 TB/s for a float4 copy). Variants, each the best of 10 launches (HIP events):
//   copy G      : grid-stride float4 copy, G blocks of 256 (fu_copy_bandwidth: G = 16384)
//   copyU G     : 4 float4 per thread per step, all loads before the stores
//   copyNT G    : as copy, non-temporal loads and stores
//   read G      : float4 loads only (a never-true store keeps them)
//   write G     : float4 stores only
//   r2w1 G      : two streams read, one written (the round kernels' mix)
// GB/s = bytes moved / device time.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_copy.hip -o tools/bin/ubench_copy
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

__global__ __launch_bounds__(256) void k_copy(const float4 *__restrict__ s, float4 *__restrict__ d, long long n) {
  const long long st = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += st) d[i] = s[i];
}

__global__ __launch_bounds__(256) void k_copyU(const float4 *__restrict__ s, float4 *__restrict__ d, long long n) {
  const long long st = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    const float4 a = s[i], b = s[i + st], c = s[i + 2 * st], e = s[i + 3 * st];
    d[i] = a;
    d[i + st] = b;
    d[i + 2 * st] = c;
    d[i + 3 * st] = e;
  }
  for (; i < n; i += st) d[i] = s[i];
}

typedef float v4f __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copyNT(const float4 *__restrict__ s4, float4 *__restrict__ d4, long long n) {
  const v4f *s = reinterpret_cast<const v4f *>(s4);
  v4f *d = reinterpret_cast<v4f *>(d4);
  const long long st = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += st)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

__global__ __launch_bounds__(256) void k_read(const float4 *__restrict__ s, long long n, float *__restrict__ out) {
  const long long st = (long long)gridDim.x * 256;
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += st) {
    const float4 x = s[i];
    acc += x.x + x.y + x.z + x.w;
  }
  if (acc == -1.2345f) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_write(float4 *__restrict__ d, long long n, float v) {
  const long long st = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += st)
    d[i] = make_float4(v, v, v, (float)(i & 7));
}

__global__ __launch_bounds__(256) void k_r2w1(const float4 *__restrict__ s0, const float4 *__restrict__ s1,
                                              float4 *__restrict__ d, long long n) {
  const long long st = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += st) {
    const float4 a = s0[i], b = s1[i];
    d[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
}

int main(int argc, char **argv) {
  const long long bytes = argc > 1 ? atoll(argv[1]) : (1ll << 29);  // per buffer
  const long long n = bytes / 16;
  float4 *a, *b, *c;
  float *out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  CK(hipMemset(c, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grids[] = {2048, 4096, 8192, 16384, 32768, 65536};
  const char *names[] = {"copy", "copyU", "copyNT", "read", "write", "r2w1"};
  for (int v = 0; v < 6; ++v) {
    for (int g : grids) {
      float best = 1e30f;
      for (int it = 0; it <= 10; ++it) {
        CK(hipEventRecord(e0, nullptr));
        switch (v) {
          case 0: hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, nullptr, a, b, n); break;
          case 1: hipLaunchKernelGGL(k_copyU, dim3(g), dim3(256), 0, nullptr, a, b, n); break;
          case 2: hipLaunchKernelGGL(k_copyNT, dim3(g), dim3(256), 0, nullptr, a, b, n); break;
          case 3: hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, nullptr, a, n, out); break;
          case 4: hipLaunchKernelGGL(k_write, dim3(g), dim3(256), 0, nullptr, b, n, (float)it); break;
          default: hipLaunchKernelGGL(k_r2w1, dim3(g), dim3(256), 0, nullptr, a, c, b, n); break;
        }
        CK(hipGetLastError());
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0 && ms < best) best = ms;
      }
      const double moved = (v == 3 || v == 4) ? (double)bytes : v == 5 ? 3.0 * bytes : 2.0 * bytes;
      printf("%-7s grid %6d  %8.1f us  %7.0f GB/s\n", names[v], g, best * 1e3, moved / (best * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
