// Single-sweep Jacobi-PCG for gfx950: ONE marching kernel and ONE global
// reduction per iteration.
//
// The reference iteration (poisson_mpi_cuda2.cu:846-942) needs two global
// reductions — (Ap,p) before α, (z,r) before β — so any implementation of it
// needs two passes over memory per iteration (the classic path here, kF+kG in
// kernels.hip, moves 8 fp64 arrays per point).  This file reorganises the
// same Krylov recurrence so that every dot product of iteration k+1 is a
// combination of dot products computable in ONE sweep over iteration k's data
// (a single-reduction CG in the spirit of Chronopoulos–Gear, but with the
// exact expansion instead of the s-recurrence, so no extra vector is kept):
//
//   p_k = z_{k-1} + β_k p_{k-1}             z = D⁻¹r
//   s_k = A p_k                              (recomputed, never stored)
//   (p_k, A p_k) = (z,Az) + 2β (z,s_{k-1}) + β² (p_{k-1},s_{k-1})
//   ‖p_k‖²        = (z,z)  + 2β (z,p_{k-1}) + β² (p_{k-1},p_{k-1})
//   α_k = (r,z)/(p_k,Ap_k),   ‖w_{k+1}-w_k‖ = |α_k| ‖p_k‖      (stop test)
//   w += α p_k,   r_k = r_{k-1} - α s_k,   z_k = D⁻¹ r_k,   q_k = A z_k
//   sums of sweep k: (r,z) (z,q) (z,s) (p,s) (z,z) (z,p) (p,p)
//
// so a sweep reads r_{k-1}, p_{k-1}, w and writes r_k, p_k, w: 6 array passes
// per point (48 B) instead of 8, and 1 reduction instead of 2 (half the
// latency-bound allreduces on multiple GPUs).  The price is a radius-2
// dependence (q needs z at ±1, z needs s at ±1, s needs p at ±1), handled by
// a 2-deep halo and by recomputation: each wave64 strip loads 128 columns but
// outputs the middle 124 (lanes 1..62), so every j-neighbour comes from a DPP
// lane shift and no strip-edge prologue is needed; rows march with the
// i-neighbours in registers and the next two rows' loads in flight.  The
// numpy prototype of this recurrence reproduces the reference's iteration
// counts exactly (tests/test_gpu.py checks the golden counts on the device).
//
// Layout: buffer x[b] interleaves the r- and p-planes by row (row stride
// `pitch` = 2 × plane width), so the two halo rows of both fields that an
// x-neighbour needs are ONE contiguous message.  Local rows -1..nx+2 and
// columns -1..ny+2 hold data (halo depth 2); everything a kernel reads past
// that is zero padding, and non-interior nodes are masked to z = 0.
#include "kcommon.hpp"

namespace pe {
namespace dev {

namespace {

constexpr int FSW = kFSW;

__device__ __forceinline__ double2 dd(double a, double b) { return make_double2(a, b); }

// Coefficients of row t for the lane's two columns: select-only when the
// strip has no boundary-band node in that row, exact face lengths otherwise.
__device__ __forceinline__ void crow(const KParams& k, const RowCls& rc, bool gen, int t, int c0, const TV& tv0,
                                     const TV& tv1, CS& x0, CS& x1) {
  if (!gen) {
    x0 = cset_fast<false>(k, rc, c0);
    x1 = cset_fast<false>(k, rc, c0 + 1);
  } else {
    x0 = cset_rc(k, rc, t, c0, tv0);
    x1 = cset_rc(k, rc, t, c0 + 1, tv1);
  }
}

__global__ __launch_bounds__(TJ) void kS(KParams k, int par) {
  DevState* st = k.st;
  if (st->done) return;
  __shared__ double sm[32];
  __shared__ int sflag;

  // ---- scalars of this sweep from the previous sweep's global sums ----
  const bool first = st->started == 0;
  const long long kiter = st->iter + 1;
  const double hh = k.h1 * k.h2;
  double alpha = 0.0, beta = 0.0, zc = 0.0, g = 0.0, diff = 0.0;
  if (!first) {
    const double* R = st->fs[par ^ 1];
    g = R[0] * hh;
    beta = st->iter == 0 ? 0.0 : g / st->gprev;
    const double den = R[1] * hh + 2.0 * beta * (R[2] * hh) + beta * beta * (R[3] * hh);
    if (fabs(den) < 1e-15) {  // breakdown: stop before touching w (reference :413)
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->status = 2;
        st->iter = kiter;
        st->done = 1;
      }
      return;
    }
    alpha = g / den;
    const double pn2 = fmax(R[4] + 2.0 * beta * R[5] + beta * beta * R[6], 0.0);
    diff = k.weighted ? fabs(alpha) * sqrt(pn2 * hh) : fabs(alpha) * sqrt(pn2);
    zc = 1.0;
  }

  const double* __restrict__ X = k.x[par ^ 1];
  double* __restrict__ Y = k.x[par];
  double* __restrict__ W = k.w;
  const int64_t pitch = k.pitch, poff = k.poff, wp = k.wpitch;
  const int nx = int(k.nx), ny = int(k.ny);
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * kWPB;
  double sg = 0.0, sd = 0.0, se = 0.0, sps = 0.0, szz = 0.0, szp = 0.0, spp = 0.0;

  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  for (int item = blockIdx.x * kWPB + wid; item < k.nitems; item += nw) {
    // chunk-major: the waves running at any moment cover a compact window of rows
    const int s = item % k.nstrips, ch = item / k.nstrips;
    const int J = -1 + s * FSW;
    const int ib = 1 + ch * k.ti, ie = min(ib + k.ti - 1, nx);
    const int c0 = J + 2 * lane;  // odd → 16-byte aligned pair (c0, c0+1)
    const int64_t g0 = k.gj0 + c0;
    const bool lv0 = c0 <= ny + 2 && g0 >= 1 && g0 <= k.N - 1;
    const bool lv1 = c0 + 1 <= ny + 2 && g0 + 1 >= 1 && g0 + 1 <= k.N - 1;
    const bool inner = lane >= 1 && lane <= 62;
    const bool o0 = inner && c0 >= 1 && c0 <= ny;
    const bool o1 = inner && c0 + 1 <= ny;
    const int jlo = J, jhi = J + 127;
    const TV tv0 = tv_at(k, c0), tv1 = tv_at(k, c0 + 1);
    // Row classes, lane t ↔ row ib-2+t.
    const int4 rcv = lane <= ie - ib + 4 ? *reinterpret_cast<const int4*>(k.rowcls + (ib - 1 + lane) * 4)
                                         : make_int4(1, 0, 0, -1);
    auto cls = [&](int t, CS& x0, CS& x1) {
      const RowCls rc = rcl_read(rcv, t - ib + 2);
      crow(k, rc, has_gen(rc, jlo, jhi), t, c0, tv0, tv1, x0, x1);
    };
    auto rlive = [&](int t) {
      const int64_t gt = k.gi0 + t;
      return gt >= 1 && gt <= k.M - 1;
    };

    const double* xr = X + int64_t(ib - 2) * pitch + c0;
    // prologue: p_k on rows ib-2, ib-1; rows ib, ib+1 queued
    const double2 rA = ld2(xr), pA = ld2(xr + poff);                          // row ib-2
    double2 rin1 = ld2(xr + pitch);                                           // row ib-1: r_{k-1}(i+1) at step i
    const double2 pB = ld2(xr + pitch + poff);
    double2 rQ0 = ld2(xr + 2 * pitch), pQ0 = ld2(xr + 2 * pitch + poff);      // row ib   (queued)
    double2 rQ1 = ld2(xr + 3 * pitch), pQ1 = ld2(xr + 3 * pitch + poff);      // row ib+1 (queued)
    xr += 4 * pitch;                                                          // → row ib+2
    double2 pa, pb;  // p_k rows i, i+1 at loop step i
    {
      CS x0, x1;
      cls(ib - 2, x0, x1);
      pa = dd(zc * (rA.x * x0.d) + beta * pA.x, zc * (rA.y * x1.d) + beta * pA.y);
      cls(ib - 1, x0, x1);
      pb = dd(zc * (rin1.x * x0.d) + beta * pB.x, zc * (rin1.y * x1.d) + beta * pB.y);
    }
    double2 wQ0 = dd(0.0, 0.0), wQ1 = dd(0.0, 0.0);
    double2 sI = dd(0.0, 0.0), rkI = dd(0.0, 0.0), zM = dd(0.0, 0.0), zI = dd(0.0, 0.0);
    const double* wr = W + int64_t(ib) * wp + c0;  // w(i+2) at step i = ib-2

    for (int i = ib - 2; i <= ie; ++i) {
      // ---- prefetch: x row i+4, w row i+2 (rows past nx+2 are padding) ----
      const double2 rN = ld2(xr), pN = ld2(xr + poff);
      const double2 wN = ld2(wr);
      xr += pitch;
      wr += wp;

      // p_k(i+2) = z_{k-1} + β p_{k-1}
      CS y0, y1;
      cls(i + 2, y0, y1);
      const double2 pc = dd(zc * (rQ0.x * y0.d) + beta * pQ0.x, zc * (rQ0.y * y1.d) + beta * pQ0.y);

      // s(i+1) = A p_k, r_k(i+1), z_k(i+1)
      CS x0, x1;
      cls(i + 1, x0, x1);
      const double pl = dpp_shr1(pb.y), pr = dpp_shl1(pb.x);
      const double s0 = stencil<false>(k, x0, pa.x, pb.x, pc.x, pl, pb.y);
      const double s1 = stencil<false>(k, x1, pa.y, pb.y, pc.y, pb.x, pr);
      const double rk0 = rin1.x - alpha * s0, rk1 = rin1.y - alpha * s1;
      const bool rl = rlive(i + 1);
      const double zn0 = (rl && lv0) ? rk0 * x0.d : 0.0;
      const double zn1 = (rl && lv1) ? rk1 * x1.d : 0.0;

      if (i >= ib) {
        // q(i) = A z_k, the 7 sums, and the row-i outputs
        CS q0c, q1c;
        cls(i, q0c, q1c);
        const double zl = dpp_shr1(zI.y), zr = dpp_shl1(zI.x);
        const double q0 = stencil<false>(k, q0c, zM.x, zI.x, zn0, zl, zI.y);
        const double q1 = stencil<false>(k, q1c, zM.y, zI.y, zn1, zI.x, zr);
        if (o0) {
          sg += rkI.x * zI.x;
          sd += zI.x * q0;
          se += zI.x * sI.x;
          sps += pa.x * sI.x;
          szz += zI.x * zI.x;
          szp += zI.x * pa.x;
          spp += pa.x * pa.x;
        }
        if (o1) {
          sg += rkI.y * zI.y;
          sd += zI.y * q1;
          se += zI.y * sI.y;
          sps += pa.y * sI.y;
          szz += zI.y * zI.y;
          szp += zI.y * pa.y;
          spp += pa.y * pa.y;
        }
        double* yr = Y + int64_t(i) * pitch + c0;
        double* wd = W + int64_t(i) * wp + c0;
        const double2 wv = dd(wQ0.x + alpha * pa.x, wQ0.y + alpha * pa.y);
        if (o1) {
          *reinterpret_cast<double2*>(yr) = rkI;
          *reinterpret_cast<double2*>(yr + poff) = pa;
          *reinterpret_cast<double2*>(wd) = wv;
        } else if (o0) {
          yr[0] = rkI.x;
          yr[poff] = pa.x;
          wd[0] = wv.x;
        }
        // y-direction halo strips (columns 1,2 and ny-1,ny) → send buffers
        if (k.has[DOWN] && o0 && c0 == 1) {
          double* sb = k.send_dn + int64_t(i - 1) * 4;
          sb[0] = rkI.x;
          sb[1] = rkI.y;
          sb[2] = pa.x;
          sb[3] = pa.y;
        }
        if (k.has[UP]) {
          double* sb = k.send_up + int64_t(i - 1) * 4;
          if (o0 && c0 >= ny - 1) {
            sb[c0 - (ny - 1)] = rkI.x;
            sb[c0 - (ny - 1) + 2] = pa.x;
          }
          if (o1 && c0 + 1 >= ny - 1) {
            sb[c0 + 1 - (ny - 1)] = rkI.y;
            sb[c0 + 1 - (ny - 1) + 2] = pa.y;
          }
        }
      }
      // ---- shift the register window ----
      zM = zI;
      zI = dd(zn0, zn1);
      sI = dd(s0, s1);
      rkI = dd(rk0, rk1);
      pa = pb;
      pb = pc;
      rin1 = rQ0;
      rQ0 = rQ1;
      pQ0 = pQ1;
      rQ1 = rN;
      pQ1 = pN;
      wQ0 = wQ1;
      wQ1 = wN;
    }
  }

  double v[7] = {sg, sd, se, sps, szz, szp, spp};
  block_reduce<7, false>(v, sm);
  if (threadIdx.x == 0)
#pragma unroll
    for (int n = 0; n < 7; ++n) k.partial[7 * size_t(blockIdx.x) + n] = v[n];
  if (arrive_last(&st->ticket[0], gridDim.x, &sflag)) {
    double t[7];
    reduce_partials<7>(k.partial, gridDim.x, t, sm);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int n = 0; n < 7; ++n) st->fs[par][n] = t[n];
      if (first) {
        st->started = 1;
      } else {
        st->gprev = g;
        st->rz_cur = g;
        st->alpha = alpha;
        st->beta = beta;
        st->last_diff = diff;
        st->iter = kiter;
        if (k.check_tol && diff < k.tol) {
          st->status = 1;
          st->done = 1;
        } else if (kiter >= k.max_iter) {
          st->status = 3;
          st->done = 1;
        }
      }
      __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// y-direction halo strips of buffer b (one thread per owned row).
__global__ void kPack(KParams k, int b) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x + 1;
  if (i > k.nx) return;
  const double* x = k.x[b] + i * k.pitch;
  if (k.has[DOWN]) {
    double* sb = k.send_dn + (i - 1) * 4;
    sb[0] = x[1];
    sb[1] = x[2];
    sb[2] = x[k.poff + 1];
    sb[3] = x[k.poff + 2];
  }
  if (k.has[UP]) {
    double* sb = k.send_up + (i - 1) * 4;
    sb[0] = x[k.ny - 1];
    sb[1] = x[k.ny];
    sb[2] = x[k.poff + k.ny - 1];
    sb[3] = x[k.poff + k.ny];
  }
}

__global__ void kUnpack(KParams k, int b) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x + 1;
  if (i > k.nx) return;
  double* x = k.x[b] + i * k.pitch;
  if (k.has[DOWN]) {
    const double* rb = k.recv_dn + (i - 1) * 4;
    x[-1] = rb[0];
    x[0] = rb[1];
    x[k.poff - 1] = rb[2];
    x[k.poff] = rb[3];
  }
  if (k.has[UP]) {
    const double* rb = k.recv_up + (i - 1) * 4;
    x[k.ny + 1] = rb[0];
    x[k.ny + 2] = rb[1];
    x[k.poff + k.ny + 1] = rb[2];
    x[k.poff + k.ny + 2] = rb[3];
  }
}

}  // namespace

void launch_S(const KParams& k, int par, hipStream_t s) {
  hipLaunchKernelGGL(kS, dim3(k.nblocks), dim3(TJ), 0, s, k, par);
}

void launch_pack(const KParams& k, int b, hipStream_t s) {
  if (!k.has[DOWN] && !k.has[UP]) return;
  hipLaunchKernelGGL(kPack, dim3(unsigned((k.nx + 255) / 256)), dim3(256), 0, s, k, b);
}

void launch_unpack(const KParams& k, int b, hipStream_t s) {
  if (!k.has[DOWN] && !k.has[UP]) return;
  hipLaunchKernelGGL(kUnpack, dim3(unsigned((k.nx + 255) / 256)), dim3(256), 0, s, k, b);
}

}  // namespace dev
}  // namespace pe
