// HBM roofline probe, second form: every lane keeps U 16-byte loads per
// array in flight before its stores (the first probe, stream_bench.hip, had
// one), plain or non-temporal stores.  R arrays read, W written, fp64.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/stream2.hip -o bin/stream2
//   bin/stream2 [doubles per array = 8192²]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ void st(v2d* p, v2d v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int R, int W, int U, bool NT>
__global__ __launch_bounds__(256) void kS(const v2d* __restrict__ a, const v2d* __restrict__ b,
                                          const v2d* __restrict__ c, v2d* __restrict__ x, v2d* __restrict__ y,
                                          v2d* __restrict__ z, long n) {
  const long S = long(gridDim.x) * 256;
  for (long i0 = blockIdx.x * 256L + threadIdx.x; i0 < n; i0 += S * U) {
    v2d va[U], vb[U], vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * S < n ? i0 + u * S : i0;
      va[u] = a[i];
      if (R > 1) vb[u] = b[i];
      if (R > 2) vc[u] = c[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * S;
      if (i >= n) break;
      v2d v = va[u];
      if (R > 1) v += vb[u];
      if (R > 2) v += vc[u];
      st<NT>(x + i, v);
      if (W > 1) st<NT>(y + i, v * 2.0);
      if (W > 2) st<NT>(z + i, v * 3.0);
    }
  }
}

int main(int argc, char** argv) {
  const long n2 = (argc > 1 ? std::atol(argv[1]) : 8192L * 8192L) / 2;
  std::vector<v2d*> p(6);
  for (auto& q : p) {
    CK(hipMalloc(&q, n2 * sizeof(v2d)));
    CK(hipMemset(q, 0, n2 * sizeof(v2d)));
  }
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, int r, int w, int u, bool nt, int bpc, auto kern) {
    const int grid = cus * bpc;
    for (int it = 0; it < 3; ++it)
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, p[0], p[1], p[2], p[3], p[4], p[5], n2);
    CK(hipEventRecord(e0));
    const int reps = 20;
    for (int it = 0; it < reps; ++it)
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, p[0], p[1], p[2], p[3], p[4], p[5], n2);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double bytes = double(r + w) * n2 * sizeof(v2d) * reps;
    std::printf("%s U=%d nt=%d blocks/CU=%d  %7.3f ms/pass  %7.1f GB/s\n", name, u, int(nt), bpc, ms / reps,
                bytes / (ms * 1e-3) / 1e9);
    std::fflush(stdout);
  };
#define RUN(R, W, U, NT, B) run(#R "R" #W "W", R, W, U, NT, B, kS<R, W, U, NT>)
  for (int b : {2, 4, 8}) {
    RUN(1, 1, 1, false, b);
    RUN(1, 1, 4, false, b);
    RUN(1, 1, 4, true, b);
    RUN(1, 1, 8, true, b);
    RUN(2, 2, 1, false, b);
    RUN(2, 2, 4, false, b);
    RUN(2, 2, 4, true, b);
    RUN(3, 3, 2, true, b);
    RUN(3, 3, 4, true, b);
  }
  return 0;
}
