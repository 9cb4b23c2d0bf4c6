// HIP runtime helpers: fail-loud error handling (reference checkCuda just
// exit()s one rank and can hang its peers — quirk A18; here the message
// names the rank/device and the process aborts, which tears down RCCL peers
// through the launcher), device selection (the reference never calls
// cudaSetDevice — quirk A5).
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "pe/device.hpp"

namespace pe {

void hip_fail(hipError_t e, const char* expr, const char* file, int line) {
  const char* rank = std::getenv("RANK");
  std::fprintf(stderr, "[pe] HIP error %d (%s) at %s:%d in `%s` (rank %s)\n", int(e), hipGetErrorString(e),
               file, line, expr, rank ? rank : "0");
  std::fflush(stderr);
  std::abort();
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Per-device pools of idle streams: solver streams and the high-priority
// halo streams of the overlap.  A new stream costs the runtime a hardware
// queue: 20-41 ms in a fresh process, the largest part of a small grid's
// construction (400×600: T_solver 0.035-0.054 s of which the stream 21-41 ms —
// PE_CTOR_TRACE=1, profiles/r4_cold.txt).  set_device() creates one of each
// while binding the process to its GPU (like the RCCL / P2P set-up, before any
// solver), one right after the other: the process has few hardware queues
// (GPU_MAX_HW_QUEUES, 4 by default) and streams take them in turn, so the
// pair gets two different queues.  (The overlap's run-to-run variance at the
// 8-rank slab of 8192² is the boundary-first sweep kernel's own duration, not
// the queues: profiles/r6_overlap_trace.txt.)  A solver returns its streams
// here when it is destroyed.
namespace {
std::mutex g_stream_mu;
std::vector<std::pair<int, hipStream_t>> g_idle_streams;  // (device, stream)
std::vector<std::pair<int, hipStream_t>> g_idle_halo;     // (device, high-priority stream)

hipStream_t take(std::vector<std::pair<int, hipStream_t>>& pool, int dev) {
  std::lock_guard<std::mutex> g(g_stream_mu);
  for (size_t i = 0; i < pool.size(); ++i)
    if (pool[i].first == dev) {
      const hipStream_t s = pool[i].second;
      pool.erase(pool.begin() + long(i));
      return s;
    }
  return nullptr;
}

void give(std::vector<std::pair<int, hipStream_t>>& pool, hipStream_t s) {
  if (!s) return;
  // filed under the device the stream was created on, not the current one (a
  // solver may be destroyed after the process moved to another device)
  hipDevice_t dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  std::lock_guard<std::mutex> g(g_stream_mu);
  pool.emplace_back(dev, s);
}
}  // namespace

static hipStream_t new_halo_stream() {
  int least = 0, greatest = 0;
  PE_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t s = nullptr;
  PE_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest));
  return s;
}

hipStream_t acquire_stream() {
  int dev = 0;
  PE_HIP_CHECK(hipGetDevice(&dev));
  if (hipStream_t s = take(g_idle_streams, dev)) return s;
  hipStream_t s = nullptr;
  PE_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // (a new solver stream gets its halo stream created right after it: the
  // pair then holds two hardware queues — see above)
  bool have_halo = false;
  {
    std::lock_guard<std::mutex> g(g_stream_mu);
    for (const auto& e : g_idle_halo) have_halo = have_halo || e.first == dev;
  }
  if (!have_halo) give(g_idle_halo, new_halo_stream());
  return s;
}

void release_stream(hipStream_t s) { give(g_idle_streams, s); }

hipStream_t acquire_halo_stream() {
  int dev = 0;
  PE_HIP_CHECK(hipGetDevice(&dev));
  if (hipStream_t s = take(g_idle_halo, dev)) return s;
  return new_halo_stream();
}

void release_halo_stream(hipStream_t s) { give(g_idle_halo, s); }

void set_device(int dev) {
  PE_HIP_CHECK(hipSetDevice(dev));
  bool have = false, have_halo = false;
  {
    std::lock_guard<std::mutex> g(g_stream_mu);
    for (const auto& e : g_idle_streams) have = have || e.first == dev;
    for (const auto& e : g_idle_halo) have_halo = have_halo || e.first == dev;
  }
  if (!have) release_stream(acquire_stream());  // (creates the halo stream next to it)
  else if (!have_halo) release_halo_stream(acquire_halo_stream());
}

int current_device() {
  int d = -1;
  PE_HIP_CHECK(hipGetDevice(&d));
  return d;
}

// "dddd:bb:dd.f" of a device: which physical GPU a rank drives (bench.py
// reports it per rank, so "N ranks on N distinct GPUs" is checkable).
std::string device_pci_bus_id(int dev) {
  char buf[64] = {0};
  PE_HIP_CHECK(hipDeviceGetPCIBusId(buf, int(sizeof buf), dev));
  return std::string(buf);
}

std::string device_name(int dev) {
  hipDeviceProp_t p;
  PE_HIP_CHECK(hipGetDeviceProperties(&p, dev));
  return std::string(p.name) + " (" + p.gcnArchName + ", " + std::to_string(p.multiProcessorCount) + " CUs, " +
         std::to_string(p.totalGlobalMem >> 30) + " GiB)";
}

}  // namespace pe
