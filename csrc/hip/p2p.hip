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

}  // namespace

void launch_p2p_sum(double* d, int n, const PeerSum& ps, hipStream_t s) {
  hipLaunchKernelGGL(kP2PSum, dim3(1), dim3(64), 0, s, d, n, ps);
}

}  // namespace dev
}  // namespace pe
