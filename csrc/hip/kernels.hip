// gfx950 (MI355X) kernels of the device-resident Jacobi-PCG solver.
//
// What the reference does per iteration (poisson_mpi_cuda2.cu:846-942):
// 5 kernels (apply_A, dot, update_w_r, apply_Dinv, dot, update_p) on a
// 16x16 block whose threadIdx.x walks the STRIDED dimension, 3 × 256 KiB of
// dot partials copied to the host and summed there, 6 device syncs, and
// a/b/B arrays streamed from HBM every time — ≈21 array passes per point.
//
// What this file does instead (8 array passes per point, 0 host syncs):
//
//   kF  (p update ⊕ stencil ⊕ 2 dots)   reads r, p_{k-1}; writes p_k
//   kG  (stop test ⊕ w,r update ⊕ recomputed stencil ⊕ (z,r) dot)
//                                        reads p_k, r, w; writes r, w
//
// Layout: row-major, j (y) contiguous, rows padded to 64 B.  A block of
// 256 threads (4 wave64s) owns a strip of 256 consecutive j and marches
// down `ti` rows of i.  Each thread keeps the i-1 / i / i+1 values of its
// own column in registers, the row's j±1 neighbours come from a
// double-buffered LDS row (one barrier per row), and the two strip-edge
// columns are produced once per block in a prologue.  The face
// coefficients a_ij, b_ij and the Jacobi diagonal D_ij are recomputed from
// two 1-D chord tables, which costs ALU (idle in this HBM-bound loop) and
// saves 3-4 array streams of HBM traffic.  Dot products end in a
// deterministic last-workgroup reduction (agent-scope release/acquire
// ticket; partials summed in block order), so results are bitwise
// reproducible run to run.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "pe/decomp.hpp"
#include "pe/problem.hpp"

namespace pe {
namespace dev {

namespace {

constexpr int TJ = kTJ;

__device__ __forceinline__ double fcoef(double l, double h, double eps, double inv_eps) {
  if (fabs(l - h) < 1e-9) return 1.0;
  if (l < 1e-9) return inv_eps;
  return (l / h) + (1.0 - l / h) / eps;
}

struct RowV {
  double sA, eA, halfB, halfB1;  // own column j: face y-range, chord of b_{·,j} and b_{·,j+1}
};

__device__ __forceinline__ RowV rowv(const KParams& k, int64_t lj) {
  const double* t = k.rowT + (lj + 1) * 4;
  RowV v;
  v.sA = t[0];
  v.eA = t[1];
  v.halfB = t[2];
  v.halfB1 = t[6];  // halfB of lj + 1
  return v;
}

// a_{q, j}: vertical face left of node q.
__device__ __forceinline__ double coefA(const KParams& k, int64_t q, const RowV& rv) {
  const double half = k.colT[(q + 1) * 4 + 0];
  return fcoef(chord_len(half, rv.sA, rv.eA), k.h2, k.eps, k.inv_eps);
}
// b_{q, j} (halfB) or b_{q, j+1} (halfB1): horizontal face below the node.
__device__ __forceinline__ double coefB(const KParams& k, int64_t q, double halfB) {
  const double sB = k.colT[(q + 1) * 4 + 1];
  const double eB = k.colT[(q + 1) * 4 + 2];
  return fcoef(chord_len(halfB, sB, eB), k.h1, k.eps, k.inv_eps);
}

template <bool EXACT>
__device__ __forceinline__ double diag(const KParams& k, double a0, double a1, double b0, double b1) {
  // D = (a_{i+1} + a_i)/h1² + (b_{j+1} + b_j)/h2²  (reference mat_D, same order)
  if constexpr (EXACT) return (a1 + a0) / k.h1sq + (b1 + b0) / k.h2sq;
  else return (a1 + a0) * (1.0 / k.h1sq) + (b1 + b0) * (1.0 / k.h2sq);
}

template <bool EXACT>
__device__ __forceinline__ double stencil(const KParams& k, double pm, double p0, double pn, double pl,
                                          double pr, double a0, double a1, double b0, double b1) {
  // Reference apply_A (poisson_mpi_cuda2.cu:526-535), same expression tree.
  if constexpr (EXACT) {
    const double Ax = k.nih1 * (a1 * (pn - p0) / k.h1 - a0 * (p0 - pm) / k.h1);
    const double Ay = k.nih2 * (b1 * (pr - p0) / k.h2 - b0 * (p0 - pl) / k.h2);
    return Ax + Ay;
  } else {
    const double Ax = (a1 * (pn - p0) - a0 * (p0 - pm)) * (-1.0 / k.h1sq);
    const double Ay = (b1 * (pr - p0) - b0 * (p0 - pl)) * (-1.0 / k.h2sq);
    return Ax + Ay;
  }
}

// Is local node (q, lj) a value this rank computes (owned, or a halo node
// whose neighbour exists)?  Global-boundary halos and halo corners are not.
__device__ __forceinline__ bool valid_node(const KParams& k, int64_t q, int64_t lj) {
  const bool rin = q >= 1 && q <= k.nx;
  const bool rh = (q == 0 && k.has[LEFT]) || (q == k.nx + 1 && k.has[RIGHT]);
  const bool cin = lj >= 1 && lj <= k.ny;
  const bool ch = (lj == 0 && k.has[DOWN]) || (lj == k.ny + 1 && k.has[UP]);
  return (rin && (cin || ch)) || (rh && cin);
}

__device__ __forceinline__ double load_r(const KParams& k, int64_t q, int64_t lj) {
  if (lj == 0) return k.recv_dn[q - 1];
  if (lj == k.ny + 1) return k.recv_up[q - 1];
  return k.r[q * k.pitch + lj];
}

template <bool EXACT>
__device__ __forceinline__ double zval(const KParams& k, double r, double D) {
  (void)k;
  return (D != 0.0) ? r / D : 0.0;
}

// Deterministic block reduction of N sums (or maxima) → thread 0.
template <int N, bool MAX>
__device__ __forceinline__ void block_reduce(double (&v)[N], double* sm) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const double t = __shfl_xor(v[n], o, 64);
      v[n] = MAX ? fmax(v[n], t) : v[n] + t;
    }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int n = 0; n < N; ++n) sm[n * 4 + wid] = v[n];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int n = 0; n < N; ++n)
      v[n] = MAX ? fmax(fmax(sm[n * 4], sm[n * 4 + 1]), fmax(sm[n * 4 + 2], sm[n * 4 + 3]))
                 : ((sm[n * 4] + sm[n * 4 + 1]) + sm[n * 4 + 2]) + sm[n * 4 + 3];
}

// Publish this block's partials and take a ticket; true in the block that
// arrives last (all partials visible to it).  Protocol: producer store →
// vmcnt(0) → agent release → vmcnt(0) → relaxed agent fetch_add; the last
// arriver does an agent acquire before reading (cdna_hip_programming §6 G16).
__device__ __forceinline__ bool arrive_last(unsigned* ticket, unsigned nblocks, int* sflag) {
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == nblocks - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *sflag = last;
  }
  __syncthreads();
  return *sflag != 0;
}

// Sum N-tuples of partials [nblocks][N] in block order (deterministic).
template <int N, bool MAX>
__device__ __forceinline__ void reduce_partials(const double* partial, unsigned nblocks, double (&v)[N],
                                                double* sm) {
#pragma unroll
  for (int n = 0; n < N; ++n) v[n] = 0.0;
  for (unsigned m = threadIdx.x; m < nblocks; m += TJ)
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const double t = partial[size_t(m) * N + n];
      v[n] = MAX ? fmax(v[n], t) : v[n] + t;
    }
  block_reduce<N, MAX>(v, sm);
}

// ---------------------------------------------------------------------------
// F: p_k = D⁻¹ r_k + β p_{k-1} on owned nodes and the halo ring, then
//    S_den = Σ (A p_k)·p_k and S_pp = Σ p_k·p_k over owned nodes.
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(TJ) void kF(KParams k, int par) {
  DevState* st = k.st;
  if (st->done) return;
  __shared__ double srow[2][TJ];
  __shared__ double hc[2][kTImax];
  __shared__ double sm[16];
  __shared__ int sflag;

  const double rz_new = (st->red_G[0] * k.h1) * k.h2;
  const double beta = rz_new / st->rz_cur;
  const double* __restrict__ pold = k.p[par ^ 1];
  double* __restrict__ pnew = k.p[par];
  const int64_t pitch = k.pitch;

  const int tx = threadIdx.x;
  const int64_t jb = int64_t(blockIdx.x) * TJ + 1;
  const int64_t lj = jb + tx;
  const int64_t ib = int64_t(blockIdx.y) * k.ti + 1;
  const int64_t ie = min(ib + int64_t(k.ti) - 1, k.nx);
  const int nrows = int(ie - ib + 1);

  // Strip-edge columns jb-1 and jb+TJ for rows ib..ie.
  if (tx < 2 * nrows) {
    const int side = tx / nrows;
    const int64_t q = ib + tx % nrows;
    const int64_t c = side ? jb + TJ : jb - 1;
    double v = 0.0;
    if (c <= k.ny + 1 && valid_node(k, q, c)) {
      const RowV rv = rowv(k, c);
      const double D = diag<EXACT>(k, coefA(k, q, rv), coefA(k, q + 1, rv), coefB(k, q, rv.halfB),
                                   coefB(k, q, rv.halfB1));
      v = zval<EXACT>(k, load_r(k, q, c), D) + beta * pold[q * pitch + c];
      if (c == 0 || c == k.ny + 1) pnew[q * pitch + c] = v;  // rank-halo column: ours to write
    }
    hc[side][tx % nrows] = v;
  }

  const bool own = lj <= k.ny;
  const bool live = lj <= k.ny + 1;
  const RowV rv = rowv(k, live ? lj : k.ny + 1);

  double a0 = coefA(k, ib, rv), a1 = coefA(k, ib + 1, rv);
  double b0 = coefB(k, ib, rv.halfB), b1 = coefB(k, ib, rv.halfB1);
  double pm = 0.0, p0 = 0.0;
  if (live) {
    if (valid_node(k, ib - 1, lj)) {
      const double D = diag<EXACT>(k, coefA(k, ib - 1, rv), a0, coefB(k, ib - 1, rv.halfB),
                                   coefB(k, ib - 1, rv.halfB1));
      pm = zval<EXACT>(k, load_r(k, ib - 1, lj), D) + beta * pold[(ib - 1) * pitch + lj];
      if (ib - 1 == 0) pnew[lj] = pm;  // rank-halo row 0
    }
    if (valid_node(k, ib, lj)) {
      const double D = diag<EXACT>(k, a0, a1, b0, b1);
      p0 = zval<EXACT>(k, load_r(k, ib, lj), D) + beta * pold[ib * pitch + lj];
      pnew[ib * pitch + lj] = p0;
    }
  }
  srow[0][tx] = p0;
  __syncthreads();

  double sden = 0.0, spp = 0.0;
  for (int64_t i = ib; i <= ie; ++i) {
    const int s = int(i - ib) & 1;
    const int64_t q = i + 1;
    const double a2 = coefA(k, q + 1, rv);
    const double bn0 = coefB(k, q, rv.halfB), bn1 = coefB(k, q, rv.halfB1);
    double pn = 0.0;
    if (live && valid_node(k, q, lj)) {
      const double D = diag<EXACT>(k, a1, a2, bn0, bn1);
      pn = zval<EXACT>(k, load_r(k, q, lj), D) + beta * pold[q * pitch + lj];
      if (q <= ie || q == k.nx + 1) pnew[q * pitch + lj] = pn;
    }
    if (own) {
      const double pl = (tx == 0) ? hc[0][i - ib] : srow[s][tx - 1];
      const double pr = (tx == TJ - 1) ? hc[1][i - ib] : srow[s][tx + 1];
      const double Ap = stencil<EXACT>(k, pm, p0, pn, pl, pr, a0, a1, b0, b1);
      sden += Ap * p0;
      spp += p0 * p0;
    }
    srow[s ^ 1][tx] = pn;
    pm = p0;
    p0 = pn;
    a0 = a1;
    a1 = a2;
    b0 = bn0;
    b1 = bn1;
    __syncthreads();
  }

  double v[2] = {sden, spp};
  block_reduce<2, false>(v, sm);
  const unsigned nb = gridDim.x * gridDim.y;
  const unsigned bid = blockIdx.y * gridDim.x + blockIdx.x;
  if (tx == 0) {
    k.partial[2 * size_t(bid)] = v[0];
    k.partial[2 * size_t(bid) + 1] = v[1];
  }
  if (arrive_last(&st->ticket[0], nb, &sflag)) {
    double t[2];
    reduce_partials<2, false>(k.partial, nb, t, sm);
    if (tx == 0) {
      st->red_F[0] = t[0];
      st->red_F[1] = t[1];
      st->rz_cur = rz_new;
      st->beta = beta;
      __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// G: α = rz/den, stop test, w += α p, r -= α A p, S_zr = Σ (D⁻¹r)·r.
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(TJ) void kG(KParams k, int par) {
  DevState* st = k.st;
  if (st->done) return;
  __shared__ double srow[2][TJ];
  __shared__ double hc[2][kTImax];
  __shared__ double sm[16];
  __shared__ int sflag;

  const double den = (st->red_F[0] * k.h1) * k.h2;
  const long long kiter = st->iter + 1;
  if (fabs(den) < 1e-15) {  // breakdown: stop before touching w (reference :413)
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
      st->status = 2;
      st->iter = kiter;
      st->done = 1;
    }
    return;
  }
  const double alpha = st->rz_cur / den;
  const double d2 = alpha * alpha * st->red_F[1];
  const double diff = k.weighted ? sqrt((d2 * k.h1) * k.h2) : sqrt(d2);

  const double* __restrict__ p = k.p[par];
  double* __restrict__ r = k.r;
  double* __restrict__ w = k.w;
  const int64_t pitch = k.pitch;
  const int tx = threadIdx.x;
  const int64_t jb = int64_t(blockIdx.x) * TJ + 1;
  const int64_t lj = jb + tx;
  const int64_t ib = int64_t(blockIdx.y) * k.ti + 1;
  const int64_t ie = min(ib + int64_t(k.ti) - 1, k.nx);
  const int nrows = int(ie - ib + 1);

  if (tx < 2 * nrows) {
    const int side = tx / nrows;
    const int64_t q = ib + tx % nrows;
    const int64_t c = side ? jb + TJ : jb - 1;
    hc[side][tx % nrows] = (c <= k.ny + 1) ? p[q * pitch + c] : 0.0;
  }
  const bool own = lj <= k.ny;
  const bool live = lj <= k.ny + 1;
  const RowV rv = rowv(k, live ? lj : k.ny + 1);
  double a0 = coefA(k, ib, rv), a1 = coefA(k, ib + 1, rv);
  double b0 = coefB(k, ib, rv.halfB), b1 = coefB(k, ib, rv.halfB1);
  double pm = live ? p[(ib - 1) * pitch + lj] : 0.0;
  double p0 = live ? p[ib * pitch + lj] : 0.0;
  srow[0][tx] = p0;
  __syncthreads();

  double szr = 0.0;
  for (int64_t i = ib; i <= ie; ++i) {
    const int s = int(i - ib) & 1;
    const int64_t q = i + 1;
    const double pn = live ? p[q * pitch + lj] : 0.0;
    const double a2 = coefA(k, q + 1, rv);
    const double bn0 = coefB(k, q, rv.halfB), bn1 = coefB(k, q, rv.halfB1);
    if (own) {
      const double pl = (tx == 0) ? hc[0][i - ib] : srow[s][tx - 1];
      const double pr = (tx == TJ - 1) ? hc[1][i - ib] : srow[s][tx + 1];
      const double Ap = stencil<EXACT>(k, pm, p0, pn, pl, pr, a0, a1, b0, b1);
      const int64_t c = i * pitch + lj;
      const double wv = w[c];
      w[c] = wv + alpha * p0;
      const double rn = r[c] - alpha * Ap;
      r[c] = rn;
      const double D = diag<EXACT>(k, a0, a1, b0, b1);
      szr += zval<EXACT>(k, rn, D) * rn;
      if (lj == 1 && k.has[DOWN]) k.send_dn[i - 1] = rn;
      if (lj == k.ny && k.has[UP]) k.send_up[i - 1] = rn;
    }
    srow[s ^ 1][tx] = pn;
    pm = p0;
    p0 = pn;
    a0 = a1;
    a1 = a2;
    b0 = bn0;
    b1 = bn1;
    __syncthreads();
  }

  double v[1] = {szr};
  block_reduce<1, false>(v, sm);
  const unsigned nb = gridDim.x * gridDim.y;
  const unsigned bid = blockIdx.y * gridDim.x + blockIdx.x;
  if (tx == 0) k.partial[bid] = v[0];
  if (arrive_last(&st->ticket[1], nb, &sflag)) {
    double t[1];
    reduce_partials<1, false>(k.partial, nb, t, sm);
    if (tx == 0) {
      st->red_G[0] = t[0];
      st->alpha = alpha;
      st->last_diff = diff;
      st->iter = kiter;
      if (k.check_tol && diff < k.tol) {
        st->status = 1;
        st->done = 1;
      } else if (kiter >= k.max_iter) {
        st->status = 3;
        st->done = 1;
      }
      __hip_atomic_store(&st->ticket[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// Init: r⁰ = B - A w⁰ (w⁰ = 0 or a global-index hash), S_zr⁰ = Σ (D⁻¹r⁰)·r⁰.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TJ) void kInit(KParams k, int init_random, unsigned long long seed, double amp) {
  __shared__ double sm[16];
  __shared__ int sflag;
  DevState* st = k.st;
  const int64_t n = k.nx * k.ny;
  double szr = 0.0;
  for (int64_t idx = int64_t(blockIdx.x) * TJ + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * TJ) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const int64_t gi = k.gi0 + li, gj = k.gj0 + lj;
    const double x = k.A1 + gi * k.h1, y = k.A2 + gj * k.h2;
    const RowV rv = rowv(k, lj);
    const double a0 = coefA(k, li, rv), a1 = coefA(k, li + 1, rv);
    const double b0 = coefB(k, li, rv.halfB), b1 = coefB(k, li, rv.halfB1);
    double rr = in_ellipse(x, y, k.cx, k.cy) ? k.F : 0.0;
    const int64_t c = li * k.pitch + lj;
    if (init_random) {
      const double w0 = random_w0(gi, gj, k.M, k.N, seed, amp);
      const double Aw = stencil<true>(k, random_w0(gi - 1, gj, k.M, k.N, seed, amp), w0,
                                      random_w0(gi + 1, gj, k.M, k.N, seed, amp),
                                      random_w0(gi, gj - 1, k.M, k.N, seed, amp),
                                      random_w0(gi, gj + 1, k.M, k.N, seed, amp), a0, a1, b0, b1);
      rr = rr - Aw;
      k.w[c] = w0;
    }
    k.r[c] = rr;
    if (lj == 1 && k.has[DOWN]) k.send_dn[li - 1] = rr;
    if (lj == k.ny && k.has[UP]) k.send_up[li - 1] = rr;
    const double D = diag<true>(k, a0, a1, b0, b1);
    szr += zval<true>(k, rr, D) * rr;
  }
  double v[1] = {szr};
  block_reduce<1, false>(v, sm);
  if (threadIdx.x == 0) k.partial[blockIdx.x] = v[0];
  if (arrive_last(&st->ticket[2], gridDim.x, &sflag)) {
    double t[1];
    reduce_partials<1, false>(k.partial, gridDim.x, t, sm);
    if (threadIdx.x == 0) {
      st->red_G[0] = t[0];
      st->rz_cur = 1.0;
      st->iter = 0;
      st->done = 0;
      st->status = 0;
      __hip_atomic_store(&st->ticket[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Error against the analytic solution u = F(1 - cx x² - cy y²)/(2cx + 2cy).
__global__ __launch_bounds__(TJ) void kError(KParams k) {
  __shared__ double sm[16];
  __shared__ int sflag;
  DevState* st = k.st;
  const int64_t n = k.nx * k.ny;
  double e2 = 0.0, emax = 0.0, omax = 0.0;
  for (int64_t idx = int64_t(blockIdx.x) * TJ + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * TJ) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const double x = k.A1 + (k.gi0 + li) * k.h1, y = k.A2 + (k.gj0 + lj) * k.h2;
    const double wv = k.w[li * k.pitch + lj];
    if (in_ellipse(x, y, k.cx, k.cy)) {
      const double e = wv - k.u_scale * (1.0 - k.cx * x * x - k.cy * y * y);
      e2 += e * e;
      emax = fmax(emax, fabs(e));
    } else {
      omax = fmax(omax, fabs(wv));
    }
  }
  double s[1] = {e2};
  double m[2] = {emax, omax};
  block_reduce<1, false>(s, sm);
  __syncthreads();
  block_reduce<2, true>(m, sm);
  if (threadIdx.x == 0) {
    k.partial[3 * size_t(blockIdx.x)] = s[0];
    k.partial[3 * size_t(blockIdx.x) + 1] = m[0];
    k.partial[3 * size_t(blockIdx.x) + 2] = m[1];
  }
  if (arrive_last(&st->ticket[3], gridDim.x, &sflag)) {
    double acc = 0.0, m0 = 0.0, m1 = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += TJ) {
      acc += k.partial[3 * size_t(b)];
      m0 = fmax(m0, k.partial[3 * size_t(b) + 1]);
      m1 = fmax(m1, k.partial[3 * size_t(b) + 2]);
    }
    double s2[1] = {acc};
    double mm[2] = {m0, m1};
    block_reduce<1, false>(s2, sm);
    __syncthreads();
    block_reduce<2, true>(mm, sm);
    if (threadIdx.x == 0) {
      st->err[0] = s2[0];
      st->err[1] = mm[0];
      st->err[2] = mm[1];
      __hip_atomic_store(&st->ticket[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void kGroupReduce(double* const* bufs, int nranks, int n, int is_max) {
  const int i = threadIdx.x;
  if (i >= n) return;
  double acc = bufs[0][i];
  for (int r = 1; r < nranks; ++r) acc = is_max ? fmax(acc, bufs[r][i]) : acc + bufs[r][i];
  for (int r = 0; r < nranks; ++r) bufs[r][i] = acc;
}

// Test op: Ap = A p on owned nodes (p halo must be valid), exact arithmetic.
__global__ void kApplyA(KParams k, const double* p, double* Ap) {
  const int64_t n = k.nx * k.ny;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const RowV rv = rowv(k, lj);
    const int64_t c = li * k.pitch + lj;
    Ap[c] = stencil<true>(k, p[c - k.pitch], p[c], p[c + k.pitch], p[c - 1], p[c + 1], coefA(k, li, rv),
                          coefA(k, li + 1, rv), coefB(k, li, rv.halfB), coefB(k, li, rv.halfB1));
  }
}

// Test op: a_ij, b_ij, D_ij on owned nodes.
__global__ void kCoef(KParams k, double* a, double* b, double* D) {
  const int64_t n = k.nx * k.ny;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const RowV rv = rowv(k, lj);
    const int64_t c = li * k.pitch + lj;
    const double a0 = coefA(k, li, rv), a1 = coefA(k, li + 1, rv);
    const double b0 = coefB(k, li, rv.halfB), b1 = coefB(k, li, rv.halfB1);
    a[c] = a0;
    b[c] = b0;
    D[c] = diag<true>(k, a0, a1, b0, b1);
  }
}

}  // namespace

int grid_blocks(const KParams& k) {
  const int64_t gx = (k.ny + TJ - 1) / TJ, gy = (k.nx + k.ti - 1) / k.ti;
  return int(gx * gy);
}

static dim3 march_grid(const KParams& k) {
  return dim3(unsigned((k.ny + TJ - 1) / TJ), unsigned((k.nx + k.ti - 1) / k.ti), 1);
}

static unsigned flat_blocks(const KParams& k) {
  const int64_t n = k.nx * k.ny;
  int64_t b = (n + TJ - 1) / TJ;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return unsigned(b);
}

void launch_init(const KParams& k, int init_random, unsigned long long seed, double amp, hipStream_t s) {
  hipLaunchKernelGGL(kInit, dim3(flat_blocks(k)), dim3(TJ), 0, s, k, init_random, seed, amp);
}

void launch_F(const KParams& k, int par, int variant, hipStream_t s) {
  if (variant == 1) hipLaunchKernelGGL(kF<false>, march_grid(k), dim3(TJ), 0, s, k, par);
  else hipLaunchKernelGGL(kF<true>, march_grid(k), dim3(TJ), 0, s, k, par);
}

void launch_G(const KParams& k, int par, int variant, hipStream_t s) {
  if (variant == 1) hipLaunchKernelGGL(kG<false>, march_grid(k), dim3(TJ), 0, s, k, par);
  else hipLaunchKernelGGL(kG<true>, march_grid(k), dim3(TJ), 0, s, k, par);
}

void launch_error(const KParams& k, hipStream_t s) {
  hipLaunchKernelGGL(kError, dim3(flat_blocks(k)), dim3(TJ), 0, s, k);
}

void launch_group_reduce(double* const* bufs, int nranks, int n, int is_max, hipStream_t s) {
  hipLaunchKernelGGL(kGroupReduce, dim3(1), dim3(64), 0, s, bufs, nranks, n, is_max);
}

void launch_apply_A(const KParams& k, const double* p, double* Ap, hipStream_t s) {
  hipLaunchKernelGGL(kApplyA, dim3(flat_blocks(k)), dim3(TJ), 0, s, k, p, Ap);
}

void launch_coef(const KParams& k, double* a, double* b, double* D, hipStream_t s) {
  hipLaunchKernelGGL(kCoef, dim3(flat_blocks(k)), dim3(TJ), 0, s, k, a, b, D);
}

}  // namespace dev
}  // namespace pe
