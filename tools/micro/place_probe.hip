// Memory-placement probe: is the single-sweep's two-speed behaviour a
// property of individual allocations (physical regions), or of how the
// sweep's concurrently streamed arrays sit relative to each other?
//
// Allocates K buffers of S bytes (default 24 × 1.07 GB = one 8192² x-plane
// pair each) and times, per buffer, an in-place read-modify-write stream and
// a read-only stream (16-B loads, 8 in flight per lane, persistent grid);
// then the sweep-like 3-array mix (read a + b, write c) over consecutive
// triples.  Prints GB/s per test; median of 5 runs each.
//
//   hipcc --offload-arch=gfx950 -O3 tools/micro/place_probe.hip -o /tmp/place_probe
//   /tmp/place_probe [K] [GB per buffer]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_rmw(v2d* a, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    v2d v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (i + u * stride < n) ? a[i + u * stride] : v2d{0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n) __builtin_nontemporal_store(v[u] * 1.0000001, a + i + u * stride);
  }
}

__global__ __launch_bounds__(256) void k_read(const v2d* a, long long n, double* out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  double s = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += 8 * stride) {
    v2d v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (i + u * stride < n) ? a[i + u * stride] : v2d{0, 0};
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u].x + v[u].y;
  }
  if (s == 12345.678) out[0] = s;
}

// sweep-like: c = a + b (two streams in, one out), 4 in flight per stream
__global__ __launch_bounds__(256) void k_mix(const v2d* a, const v2d* b, v2d* c, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    v2d x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool in = i + u * stride < n;
      x[u] = in ? a[i + u * stride] : v2d{0, 0};
      y[u] = in ? b[i + u * stride] : v2d{0, 0};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n) __builtin_nontemporal_store(x[u] + y[u], c + i + u * stride);
  }
}

template <class F>
static float timed(F&& f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  f();
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return t[2];
}

// Mode "offsets": ONE allocation (plain, or physically contiguous) holding
// the three arrays at base, base + S + d, base + 2S + 2d, for a range of d —
// if the speed is set by the arrays' relative physical offsets, it shows here.
static int offsets_mode(int contiguous, double gb) {
  const size_t S = size_t(gb * 1e9) / 4096 * 4096;
  const long long n = (long long)(S / 16);
  const size_t dmax = size_t(64) << 20;
  const size_t total = 3 * S + 2 * dmax + (size_t(4) << 20);
  char* base = nullptr;
  if (contiguous) CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&base), total, hipDeviceMallocContiguous));
  else CK(hipMalloc(&base, total));
  CK(hipMemset(base, 0, total));
  CK(hipDeviceSynchronize());
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 8;
  std::printf("# one %s allocation, arrays at 0, S+d, 2S+2d (S = %.3f GB); mix GB/s (3 x bytes)\n",
              contiguous ? "contiguous" : "plain", double(S) / 1e9);
  const size_t ds[] = {0, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536, 131072, 262144, 524288,
                       size_t(1) << 20, size_t(2) << 20, size_t(3) << 20, size_t(4) << 20, size_t(6) << 20,
                       size_t(8) << 20, size_t(12) << 20, size_t(16) << 20, size_t(24) << 20, size_t(32) << 20,
                       size_t(48) << 20, size_t(64) << 20};
  for (size_t d : ds) {
    const v2d* a = reinterpret_cast<const v2d*>(base);
    const v2d* b = reinterpret_cast<const v2d*>(base + S + d);
    v2d* c = reinterpret_cast<v2d*>(base + 2 * S + 2 * d);
    const float t = timed([&] { hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, a, b, c, n); });
    std::printf("d = %9zu B: %6.0f\n", d, 3.0 * double(S) / (t * 1e6));
    std::fflush(stdout);
  }
  CK(hipFree(base));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "offsets")
    return offsets_mode(argc > 2 ? std::atoi(argv[2]) : 0, argc > 3 ? std::atof(argv[3]) : 1.074);
  const int K = argc > 1 ? std::atoi(argv[1]) : 24;
  const double gb = argc > 2 ? std::atof(argv[2]) : 1.074;
  const size_t bytes = size_t(gb * 1e9) / 4096 * 4096;
  const long long n = (long long)(bytes / 16);
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 8;
  std::vector<v2d*> buf(size_t(K), nullptr);
  for (int i = 0; i < K; ++i) {
    CK(hipMalloc(&buf[size_t(i)], bytes));
    CK(hipMemset(buf[size_t(i)], 0, bytes));
  }
  double* out = nullptr;
  CK(hipMalloc(&out, 8));
  CK(hipDeviceSynchronize());
  std::printf("# %d buffers x %.3f GB; GB/s (median of 5): rmw = 2 x bytes, read = bytes, mix(i,i+1->i+2) = 3 x bytes\n", K,
              double(bytes) / 1e9);
  std::printf("%4s %14s %8s %8s %10s\n", "buf", "vaddr", "rmw", "read", "mix");
  for (int i = 0; i < K; ++i) {
    v2d* a = buf[size_t(i)];
    const float t_rmw = timed([&] { hipLaunchKernelGGL(k_rmw, dim3(grid), dim3(256), 0, 0, a, n); });
    const float t_rd = timed([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, out); });
    float t_mix = 0.f;
    if (i + 2 < K) {
      v2d *b = buf[size_t(i + 1)], *c = buf[size_t(i + 2)];
      t_mix = timed([&] { hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, a, b, c, n); });
    }
    std::printf("%4d %14p %8.0f %8.0f %10.0f\n", i, (void*)a, 2.0 * double(bytes) / (t_rmw * 1e6),
                double(bytes) / (t_rd * 1e6), t_mix > 0 ? 3.0 * double(bytes) / (t_mix * 1e6) : 0.0);
    std::fflush(stdout);
  }
  for (auto* p : buf) CK(hipFree(p));
  return 0;
}
