// One-shot peer-to-peer allreduce of a few doubles over xGMI.
//
// The reference's per-iteration global sums are 8-byte MPI_Allreduce calls
// preceded by a device sync (poisson_mpi_cuda2.cu:842, :871, :892, :925;
// SURVEY C26).  This kernel instead writes the local vector straight into a
// slot of every peer's receive buffer (fine-grained memory, IPC-mapped over
// xGMI) and sums the P slots of its own buffer in rank order (protocol:
// peer_sum.hpp).  The single-sweep solver does the same exchange inside its
// final reduction block (KParams::xr), so it only launches this kernel for
// the other, rare collectives (error norms, tests).
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "peer_sum.hpp"

namespace pe {
namespace dev {
namespace {

__global__ void kP2PSum(double* d, int n, PeerSum ps) {
  __shared__ double v[kP2PSlot];
  __shared__ unsigned long long sseq;
  __shared__ int sok;
  if (int(threadIdx.x) < n) v[threadIdx.x] = d[threadIdx.x];
  __syncthreads();
  peer_sum_block(ps, v, n, &sseq, &sok);
  if (int(threadIdx.x) < n) d[threadIdx.x] = v[threadIdx.x];
}

// d[i] = s[i] for i in [lo, hi) by the block (NaN with `poison`): 16-byte
// accesses when s and d share their 16-byte phase (the x rows of a halo: the
// inbox slot is offset by one double so that it matches them), 8-byte
// otherwise; 4 loads in flight per lane before their stores (the remote
// stores are write-through: the copy is bound by how many are outstanding).
__device__ __forceinline__ void copy_span(const double* __restrict__ s, double* __restrict__ d, long long lo,
                                          long long hi, bool poison) {
  const int T = int(blockDim.x), t = int(threadIdx.x);
  const double nan = __builtin_nan("");
  if (((reinterpret_cast<uintptr_t>(s) ^ reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
    long long a = lo;
    if (a < hi && (reinterpret_cast<uintptr_t>(s + a) & 15)) {
      if (t == 0) d[a] = poison ? nan : s[a];
      ++a;
    }
    const long long np = (hi - a) / 2;
    const double2* s2 = reinterpret_cast<const double2*>(s + a);
    double2* d2 = reinterpret_cast<double2*>(d + a);
    const double2 n2 = make_double2(nan, nan);
    long long k = t;
    for (; k + 3 * T < np; k += 4 * T) {
      double2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = s2[k + u * T];
#pragma unroll
      for (int u = 0; u < 4; ++u) d2[k + u * T] = poison ? n2 : v[u];
    }
    for (; k < np; k += T) d2[k] = poison ? n2 : s2[k];
    if (((hi - a) & 1) && t == 0) d[hi - 1] = poison ? nan : s[hi - 1];
    return;
  }
  long long i = lo + t;
  for (; i + 3 * T < hi; i += 4 * T) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = s[i + u * T];
#pragma unroll
    for (int u = 0; u < 4; ++u) d[i + u * T] = poison ? nan : v[u];
  }
  for (; i < hi; i += T) d[i] = poison ? nan : s[i];
}

// Halo exchange by peer put (protocol: kernels.hpp PutArgs).  Block
// (part b, message m): b = blockIdx / nmsg, so every message's part 0 is
// dispatched before any part 1 — each block waits only for the SAME part of
// its peer's message, and the in-order dispatch on both GPUs then guarantees
// progress with as few as nmsg resident blocks (the overlap keeps 8 free).
// Element i of a message sits at inbox[parity][1 + i] (kPutBoxOff).
__global__ __launch_bounds__(256) void kPut(PutArgs a) {
  const int m = int(blockIdx.x) % a.nmsg, b = int(blockIdx.x) / a.nmsg;
  const PutMsg g = a.m[m];
  __shared__ unsigned long long sc;
  __shared__ int sok;
  if (threadIdx.x == 0) {
    sc = __hip_atomic_load(a.cnt + g.dir, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sok = 1;
  }
  __syncthreads();
  const unsigned long long c = sc;
  const long long par = (long long)(c & 1ull) * a.stride + kPutBoxOff;
  const long long lo = g.n * b / a.parts, hi = g.n * (b + 1) / a.parts;
  copy_span(g.src, g.rbox + par, lo, hi, false);
  // Every wave's stores complete (performed at its XCD's L2, or beyond for
  // the uncached fine-grained memory) before the flag; the flag's one
  // system-scope release then writes that L2 back — one writeback per block,
  // not one per wave (a release fence in every wave cost each wave an L2
  // writeback).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(g.rflag + size_t(b) * kPutFlagStride, c + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long* f = g.lflag + size_t(b) * kPutFlagStride;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < c + 1) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
        sok = 0;  // the peer never arrived: poison instead of hanging
        break;
      }
    }
    // one acquire for the block: it invalidates this CU's L1 and its XCD's
    // L2, which every wave of the block reads the inbox through
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  copy_span(g.lbox + par, g.dst, lo, hi, sok == 0);
  __syncthreads();
  if (threadIdx.x == 0) {
    // the message's last part advances the direction's count (every part read
    // it above, before its ticket)
    const unsigned t = __hip_atomic_fetch_add(a.cnt + 4 + g.dir, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == unsigned(a.parts - 1)) {
      __hip_atomic_store(a.cnt + 4 + g.dir, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.cnt + g.dir, unsigned(c + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(256) void kPutCheck(PutArgs a, const double* codes, int* bad) {
  const int m = int(blockIdx.x);
  if (m >= a.nmsg) return;
  const PutMsg g = a.m[m];
  int nb = 0;
  for (long long i = threadIdx.x; i < g.n; i += blockDim.x) nb += g.dst[i] != codes[m] + double(i % 7);
  if (nb) atomicAdd(bad, nb);
}

}  // namespace

void launch_put(const PutArgs& a, hipStream_t s) {
  if (a.nmsg <= 0) return;
  hipLaunchKernelGGL(kPut, dim3(unsigned(a.nmsg * a.parts)), dim3(256), 0, s, a);
}

void launch_put_check(const PutArgs& a, const double* codes, int* bad, hipStream_t s) {
  if (a.nmsg <= 0) return;
  hipLaunchKernelGGL(kPutCheck, dim3(unsigned(a.nmsg)), dim3(256), 0, s, a, codes, bad);
}

void launch_p2p_sum(double* d, int n, const PeerSum& ps, hipStream_t s) {
  hipLaunchKernelGGL(kP2PSum, dim3(1), dim3(64), 0, s, d, n, ps);
}

}  // namespace dev
}  // namespace pe
