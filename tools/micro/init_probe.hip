// First-use costs of the HIP runtime calls a solver construction makes, in
// a fresh process after device selection (which the timers exclude, as the
// reference's time_solver excludes MPI_Init): which of them dominate the
// ≈40 ms construction of the small published grids?
//
//   hipcc --offload-arch=gfx950 -O3 tools/micro/init_probe.hip -o tools/micro/init_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

__global__ void k_fill(double* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = double(i);
}
__global__ void k_copy(const double* __restrict__ src, double* dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

#define T(label, stmt)                                              \
  do {                                                              \
    const auto t0 = clk::now();                                     \
    stmt;                                                           \
    (void)hipDeviceSynchronize();                                   \
    std::printf("%-44s %9.3f ms\n", label, ms_since(t0));           \
  } while (0)

int main() {
  int n = 0;
  T("hipGetDeviceCount", (void)hipGetDeviceCount(&n));
  T("hipSetDevice(0)", (void)hipSetDevice(0));
  hipDeviceProp_t prop;
  T("hipGetDeviceProperties", (void)hipGetDeviceProperties(&prop, 0));
  double *a = nullptr, *b = nullptr, *c = nullptr, *h = nullptr;
  T("hipMalloc 1 MB (first)", (void)hipMalloc(&a, 1 << 20));
  T("hipMalloc 1 MB (second)", (void)hipMalloc(&b, 1 << 20));
  T("hipMalloc 1 GB", (void)hipMalloc(&c, size_t(1) << 30));
  T("kernel launch on hipStreamPerThread (first)",
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, hipStreamPerThread, a, 1 << 14));
  T("kernel launch on hipStreamPerThread (second)",
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, hipStreamPerThread, a, 1 << 14));
  {
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    const hipError_t e0 = hipStreamBeginCapture(hipStreamPerThread, hipStreamCaptureModeThreadLocal);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, hipStreamPerThread, a, 1 << 14);
    const hipError_t e1 = hipStreamEndCapture(hipStreamPerThread, &g);
    const hipError_t e2 = g ? hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) : hipErrorInvalidValue;
    std::printf("capture on hipStreamPerThread: begin %d end %d instantiate %d\n", int(e0), int(e1), int(e2));
    (void)hipGetLastError();
  }
  hipStream_t s0;
  T("hipStreamCreate (first)", (void)hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  T("kernel launch on it (first)", hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, s0, a, 1 << 14));
  double* hp = nullptr;
  T("hipHostMalloc 1 MB pinned (first)", (void)hipHostMalloc(&hp, 1 << 20, hipHostMallocDefault));
  T("kernel writes pinned host memory (first)", hipLaunchKernelGGL(k_copy, dim3(64), dim3(256), 0, s0, a, hp, 1 << 14));
  T("kernel writes pinned host memory (second)", hipLaunchKernelGGL(k_copy, dim3(64), dim3(256), 0, s0, a, hp, 1 << 14));
  T("kernel reads pinned host memory (first)", hipLaunchKernelGGL(k_copy, dim3(64), dim3(256), 0, s0, hp, b, 1 << 14));
  hipEvent_t e0, e1;
  T("hipEventCreate x2", ((void)hipEventCreate(&e0), (void)hipEventCreate(&e1)));
  T("hipEventRecord + sync", ((void)hipEventRecord(e0, s0), (void)hipEventRecord(e1, s0), (void)hipEventSynchronize(e1)));
  float ms = 0;
  T("hipEventElapsedTime", (void)hipEventElapsedTime(&ms, e0, e1));
  T("hipMemcpyAsync D2H 8 B pinned on stream (first copy)", ((void)hipMemcpyAsync(hp, a, 8, hipMemcpyDeviceToHost, s0), (void)hipStreamSynchronize(s0)));
  T("hipMemcpyAsync D2H 8 B pinned on stream (second)", ((void)hipMemcpyAsync(hp, a, 8, hipMemcpyDeviceToHost, s0), (void)hipStreamSynchronize(s0)));
  std::vector<double> host(1 << 14, 1.0);
  T("hipMemcpy H2D 128 KB pageable (first)", (void)hipMemcpy(a, host.data(), host.size() * 8, hipMemcpyHostToDevice));
  T("hipMemcpy H2D 128 KB pageable (second)", (void)hipMemcpy(b, host.data(), host.size() * 8, hipMemcpyHostToDevice));
  T("hipHostMalloc 128 KB pinned", (void)hipHostMalloc(&h, host.size() * 8, hipHostMallocDefault));
  for (size_t i = 0; i < host.size(); ++i) h[i] = 2.0;
  T("hipMemcpy H2D 128 KB pinned", (void)hipMemcpy(a, h, host.size() * 8, hipMemcpyHostToDevice));
  T("kernel launch (first)", hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, a, 1 << 14));
  T("kernel launch (second)", hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, a, 1 << 14));
  T("kernel reads pinned host memory", hipLaunchKernelGGL(k_copy, dim3(64), dim3(256), 0, 0, h, b, 1 << 14));
  T("hipMemset 1 GB", (void)hipMemset(c, 0, size_t(1) << 30));
  T("hipMemcpy D2H 128 KB pageable", (void)hipMemcpy(host.data(), a, host.size() * 8, hipMemcpyDeviceToHost));
  T("hipMemcpy D2H 128 KB pinned", (void)hipMemcpy(h, a, host.size() * 8, hipMemcpyDeviceToHost));
  hipStream_t s;
  T("hipStreamCreate", (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  T("hipMemcpyAsync H2D pageable on new stream",
    (void)hipMemcpyAsync(a, host.data(), host.size() * 8, hipMemcpyHostToDevice, s));
  return 0;
}
