// HBM roofline probe for MI355X: fp64 streams with the single-sweep PCG
// kernel's traffic mix (3 arrays read + 3 written per point) and simpler
// mixes, grid-stride, 16-byte accesses.  Prints GB/s per pattern.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/stream_bench.hip -o bin/stream_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

template <int R, int W>
__global__ __launch_bounds__(256) void kStream(const double2* __restrict__ a, const double2* __restrict__ b,
                                               const double2* __restrict__ c, double2* __restrict__ x,
                                               double2* __restrict__ y, double2* __restrict__ z, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256) {
    double2 v = a[i];
    if (R > 1) {
      const double2 t = b[i];
      v.x += t.x;
      v.y += t.y;
    }
    if (R > 2) {
      const double2 t = c[i];
      v.x += t.x;
      v.y += t.y;
    }
    x[i] = v;
    if (W > 1) y[i] = make_double2(v.y, v.x);
    if (W > 2) z[i] = make_double2(v.x * 2.0, v.y);
  }
}

int main(int argc, char** argv) {
  const long n2 = (argc > 1 ? std::atol(argv[1]) : 8192L * 8192L) / 2;  // double2 elements per array
  const int mode = argc > 2 ? std::atoi(argv[2]) : 0;  // 0 separate hipMalloc, 1 one slab, 2 one contiguous slab
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 1;
  for (int round = 0; round < rounds; ++round) {
  std::vector<double2*> p(6);
  void* slab = nullptr;
  if (mode == 0) {
    for (auto& q : p) CK(hipMalloc(&q, n2 * sizeof(double2)));
  } else {
    const size_t bytes = 6 * n2 * sizeof(double2);
    if (mode == 2) CK(hipExtMallocWithFlags(&slab, bytes, hipDeviceMallocContiguous));
    else CK(hipMalloc(&slab, bytes));
    for (int i = 0; i < 6; ++i) p[i] = static_cast<double2*>(slab) + i * n2;
  }
  for (auto& q : p) CK(hipMemset(q, 0, n2 * sizeof(double2)));
  std::printf("round %d mode %d base %p\n", round, mode, (void*)p[0]);
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, int r, int w, auto kern) {
    for (int blocks_per_cu : {8}) {
      const int grid = cus * blocks_per_cu;
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
      const double bytes = double(r + w) * n2 * sizeof(double2) * reps;
      std::printf("%-8s grid=%5d  %7.3f ms/pass  %7.1f GB/s\n", name, grid, ms / reps, bytes / (ms * 1e-3) / 1e9);
    }
  };
  run("1R1W", 1, 1, kStream<1, 1>);
  run("2R1W", 2, 1, kStream<2, 1>);
  run("3R3W", 3, 3, kStream<3, 3>);
  run("3R2W", 3, 2, kStream<3, 2>);
  (void)slab;  // kept: later rounds get fresh placements
  }
  return 0;
}
