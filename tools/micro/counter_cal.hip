// Calibration of the DRAM request counters: kernels that
// move a KNOWN number of bytes in the access widths the three-step sweep
// uses, so TCC_EA0_RDREQ / TCC_EA0_WRREQ (and FETCH_SIZE / WRITE_SIZE) can be
// converted to bytes with evidence instead of an assumed 128 B / 64 B per
// request.  Every array is 1 GiB (4× the 256 MiB Infinity Cache, so re-use
// across dispatches cannot be served on-die) and each kernel is launched
// 3 times; the per-dispatch counters divided by the logical bytes give bytes
// per request.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/counter_cal.hip -o bin/counter_cal
//   rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -- bin/counter_cal
// Kernels (each wave touches whole 128-B lines unless named otherwise):
//   kRead8     8 B / lane plain loads (the sweep's r, p loads)          read N
//   kRead8nt   8 B / lane non-temporal loads (the sweep's w loads)      read N
//   kRead16    16 B / lane plain loads                                  read N
//   kCopy8nt   8 B / lane plain load + non-temporal store (r, p, w out) read N, write N
//   kCopy16    16 B / lane load + store                                 read N, write N
//   kWrite8nt  8 B / lane non-temporal stores only                      write N
//   kStrip     the sweep's strip geometry: per row, 64 lanes load 512 B
//              (4 aligned lines), lanes 8..55 store 384 B (6 aligned 64-B
//              segments); strips 48 columns apart share a 128-B line of
//              halo with each neighbour: read ≈ 64/48 N', write N'
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void kRead8(const double* __restrict__ a, double* sink, long n) {
  double acc = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256) acc += a[i];
  if (acc == 1.2345e300) sink[0] = acc;  // (never true: keeps the loads)
}

__global__ __launch_bounds__(256) void kRead8nt(const double* __restrict__ a, double* sink, long n) {
  double acc = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256)
    acc += __builtin_nontemporal_load(a + i);
  if (acc == 1.2345e300) sink[0] = acc;
}

__global__ __launch_bounds__(256) void kRead16(const v2d* __restrict__ a, double* sink, long n2) {
  v2d acc = {0.0, 0.0};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n2; i += long(gridDim.x) * 256) acc += a[i];
  if (acc.x + acc.y == 1.2345e300) sink[0] = acc.x;
}

__global__ __launch_bounds__(256) void kCopy8nt(const double* __restrict__ a, double* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256)
    __builtin_nontemporal_store(a[i] * 2.0, y + i);
}

__global__ __launch_bounds__(256) void kCopy16(const v2d* __restrict__ a, v2d* __restrict__ y, long n2) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n2; i += long(gridDim.x) * 256) y[i] = a[i] * 2.0;
}

__global__ __launch_bounds__(256) void kWrite8nt(double* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256)
    __builtin_nontemporal_store(double(i), y + i);
}

// One wave per (strip, row) task; pitch a multiple of 16 doubles (128 B).
__global__ __launch_bounds__(256) void kStrip(const double* __restrict__ a, double* __restrict__ y, long pitch,
                                              int strips, long rows) {
  const int lane = threadIdx.x & 63;
  const long nw = long(gridDim.x) * 4, ntask = long(strips) * rows;
  for (long t = blockIdx.x * 4L + (threadIdx.x >> 6); t < ntask; t += nw) {
    const long row = t / strips;
    const int s = int(t - row * strips);
    const long o = row * pitch + 48L * s + lane;
    const double v = a[o];
    if (lane >= 8 && lane < 56) __builtin_nontemporal_store(v * 2.0, y + o);
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : (1L << 27);  // doubles per array: 1 GiB
  double *a = nullptr, *y = nullptr, *sink = nullptr;
  CK(hipMalloc(&a, sizeof(double) * n));
  CK(hipMalloc(&y, sizeof(double) * n));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, sizeof(double) * n));
  CK(hipMemset(y, 0, sizeof(double) * n));
  int ncu = 256;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const dim3 g(unsigned(ncu * 8)), b(256);
  // strip geometry: 171 strips (8192 columns), pitch = 48·171 + 16 rounded to 16
  const int strips = 171;
  const long pitch = ((48L * strips + 16 + 15) / 16) * 16;
  const long rows = n / pitch - 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double rd, double wr, auto launch) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("%-10s rep %d  logical read %.6e B  write %.6e B  %.3f ms  %.2f TB/s\n", name, rep, rd, wr, ms,
                  (rd + wr) / (ms * 1e-3) / 1e12);
    }
  };
  const double B = 8.0 * double(n);
  run("kRead8", B, 0, [&] { hipLaunchKernelGGL(kRead8, g, b, 0, 0, a, sink, n); });
  run("kRead8nt", B, 0, [&] { hipLaunchKernelGGL(kRead8nt, g, b, 0, 0, a, sink, n); });
  run("kRead16", B, 0, [&] { hipLaunchKernelGGL(kRead16, g, b, 0, 0, reinterpret_cast<const v2d*>(a), sink, n / 2); });
  run("kCopy8nt", B, B, [&] { hipLaunchKernelGGL(kCopy8nt, g, b, 0, 0, a, y, n); });
  run("kCopy16", B, B,
      [&] { hipLaunchKernelGGL(kCopy16, g, b, 0, 0, reinterpret_cast<const v2d*>(a), reinterpret_cast<v2d*>(y), n / 2); });
  run("kWrite8nt", 0, B, [&] { hipLaunchKernelGGL(kWrite8nt, g, b, 0, 0, y, n); });
  // strip: unique lines read = rows × (48·strips + 16) columns (each line once
  // if the shared halo lines hit L2 / MALL), loads issued = rows × 64·strips
  const double srd_unique = 8.0 * double(rows) * (48.0 * strips + 16.0);
  const double srd_issued = 8.0 * double(rows) * 64.0 * strips;
  const double swr = 8.0 * double(rows) * 48.0 * strips;
  std::printf("kStrip geometry: rows %ld strips %d pitch %ld: read unique %.6e B, issued %.6e B\n", rows, strips, pitch,
              srd_unique, srd_issued);
  run("kStrip", srd_unique, swr, [&] { hipLaunchKernelGGL(kStrip, g, b, 0, 0, a, y, pitch, strips, rows); });
  CK(hipDeviceSynchronize());
  std::printf("DONE\n");
  return 0;
}
