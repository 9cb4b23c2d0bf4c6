// HBM ceiling on this MI355X: what the best streaming code achieves, as the
// anchor for "% of roofline" claims (docs/PERFORMANCE.md).  Three references:
//   * hipMemcpyDtoD (the runtime's copy engine / blit kernel),
//   * best-effort R-read / W-write fp64 stream kernels (16-B accesses), swept
//     over blocks per CU, loads in flight per lane (U) and non-temporal
//     stores — R,W = 1,0 (read-only), 1,1, 2,2, 3,3 (the single sweep's
//     mix: r, p, w in and out),
//   * each at several allocations (placement changes the rate, see
//     docs/PERFORMANCE.md "Memory placement"): best and median reported.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/roofline.hip -o bin/roofline
//   bin/roofline [doubles per array = 8192²] [allocations = 4]
#include <hip/hip_runtime.h>

#include <algorithm>
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

template <int R, int W, int U, bool NT>
__global__ __launch_bounds__(256) void kStream(const v2d* __restrict__ a, const v2d* __restrict__ b,
                                               const v2d* __restrict__ c, v2d* __restrict__ x, v2d* __restrict__ y,
                                               v2d* __restrict__ z, v2d* __restrict__ sink, long n) {
  const long S = long(gridDim.x) * 256;
  v2d acc = {0.0, 0.0};
  for (long i0 = blockIdx.x * 256L + threadIdx.x; i0 < n; i0 += S * U) {
    v2d va[U], vb[U], vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * S < n ? i0 + u * S : i0;
      va[u] = __builtin_nontemporal_load(a + i);
      if (R > 1) vb[u] = __builtin_nontemporal_load(b + i);
      if (R > 2) vc[u] = __builtin_nontemporal_load(c + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * S;
      if (i >= n) break;
      v2d v = va[u];
      if (R > 1) v += vb[u];
      if (R > 2) v += vc[u];
      if (W == 0) acc += v;
      if (W > 0) {
        if (NT) __builtin_nontemporal_store(v, x + i);
        else x[i] = v;
      }
      if (W > 1) {
        if (NT) __builtin_nontemporal_store(v, y + i);
        else y[i] = v;
      }
      if (W > 2) {
        if (NT) __builtin_nontemporal_store(v, z + i);
        else z[i] = v;
      }
    }
  }
  if (W == 0 && acc.x == 12345.678) sink[0] = acc;  // keeps the loads live
}

struct Bufs {
  v2d *a, *b, *c, *x, *y, *z, *sink;
};

template <int R, int W, int U, bool NT>
float run(const Bufs& B, long n, int blocks, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((kStream<R, W, U, NT>), dim3(blocks), dim3(256), 0, 0, B.a, B.b, B.c, B.x, B.y, B.z, B.sink, n);
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((kStream<R, W, U, NT>), dim3(blocks), dim3(256), 0, 0, B.a, B.b, B.c, B.x, B.y, B.z, B.sink,
                       n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / reps;
}

struct Row {
  const char* name;
  std::vector<double> gbs;  // per allocation: the best over the configuration sweep
  std::vector<int> cfg_bpc, cfg_u, cfg_nt;
};

int main(int argc, char** argv) {
  const long nd = argc > 1 ? std::atol(argv[1]) : 8192L * 8192L;
  const int nalloc = argc > 2 ? std::atoi(argv[2]) : 4;
  const long n = nd / 2;  // v2d elements
  const size_t bytes = sizeof(double) * size_t(nd);
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::printf("# %ld doubles (%.0f MiB) per array, %d CUs, %d allocations\n", nd, bytes / 1048576.0, cus, nalloc);
  std::vector<double> memcpy_gbs;
  struct Pat {
    const char* name;
    int R, W;
  };
  const Pat pats[] = {{"1R0W", 1, 0}, {"1R1W", 1, 1}, {"2R2W", 2, 2}, {"3R3W", 3, 3}};
  std::vector<std::vector<double>> best(4);
  std::vector<std::vector<int>> bcfg(4);
  std::vector<void*> spacers;
  for (int al = 0; al < nalloc; ++al) {
    if (al > 0) {  // a spacer between candidates so they land elsewhere
      void* sp = nullptr;
      if (hipMalloc(&sp, size_t(4) << 30) == hipSuccess) spacers.push_back(sp);
    }
    Bufs B{};
    CK(hipMalloc(&B.a, bytes));
    CK(hipMalloc(&B.b, bytes));
    CK(hipMalloc(&B.c, bytes));
    CK(hipMalloc(&B.x, bytes));
    CK(hipMalloc(&B.y, bytes));
    CK(hipMalloc(&B.z, bytes));
    CK(hipMalloc(&B.sink, 64));
    for (v2d* p : {B.a, B.b, B.c, B.x, B.y, B.z}) CK(hipMemset(p, 0, bytes));
    // copy engine
    {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipMemcpy(B.x, B.a, bytes, hipMemcpyDeviceToDevice));
      CK(hipEventRecord(e0));
      for (int r = 0; r < 10; ++r) CK(hipMemcpyAsync(B.x, B.a, bytes, hipMemcpyDeviceToDevice, 0));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      memcpy_gbs.push_back(2.0 * bytes / (ms / 10 * 1e-3) / 1e9);
    }
    for (int pi = 0; pi < 4; ++pi) {
      double bestv = 0;
      int bb = 0, bu = 0, bn = 0;
      for (int bpc : {1, 2, 4, 8, 16}) {
        const int blocks = bpc * cus;
        for (int u : {1, 4, 8}) {
          for (int nt = 0; nt < 2; ++nt) {
            if (pats[pi].W == 0 && nt) continue;
            float ms = 0;
            const int R = pats[pi].R, W = pats[pi].W;
#define CASE(RR, WW, UU)                                                              \
  if (R == RR && W == WW && u == UU)                                                  \
    ms = nt ? run<RR, WW, UU, true>(B, n, blocks, 8) : run<RR, WW, UU, false>(B, n, blocks, 8);
            CASE(1, 0, 1) CASE(1, 0, 4) CASE(1, 0, 8) CASE(1, 1, 1) CASE(1, 1, 4) CASE(1, 1, 8)
            CASE(2, 2, 1) CASE(2, 2, 4) CASE(2, 2, 8) CASE(3, 3, 1) CASE(3, 3, 4) CASE(3, 3, 8)
#undef CASE
            const double gbs = double(R + W) * bytes / (ms * 1e-3) / 1e9;
            if (gbs > bestv) {
              bestv = gbs;
              bb = bpc;
              bu = u;
              bn = nt;
            }
          }
        }
      }
      best[pi].push_back(bestv);
      bcfg[pi].push_back(bb * 100 + bu * 10 + bn);
      std::printf("alloc %d  %s best %7.1f GB/s  (blocks/CU %d, U %d, nt %d)\n", al, pats[pi].name, bestv, bb, bu, bn);
      std::fflush(stdout);
    }
    std::printf("alloc %d  hipMemcpyDtoD %7.1f GB/s (read + write)\n", al, memcpy_gbs.back());
    for (v2d* p : {B.a, B.b, B.c, B.x, B.y, B.z, B.sink}) CK(hipFree(p));
  }
  for (void* sp : spacers) CK(hipFree(sp));
  auto summary = [](const char* name, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    std::printf("SUMMARY %-14s best %7.1f  median %7.1f  worst %7.1f GB/s\n", name, v.back(), v[v.size() / 2], v[0]);
  };
  summary("hipMemcpyDtoD", memcpy_gbs);
  for (int pi = 0; pi < 4; ++pi) summary(pats[pi].name, best[pi]);
  return 0;
}
