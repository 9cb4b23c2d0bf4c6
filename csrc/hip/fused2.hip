// Two-step single sweep: TWO Jacobi-PCG iterations per pass over memory.
//
// fused.hip's single sweep needs one pass per iteration because the scalars
// of iteration k+1 depend on dot products of iteration k's vectors.  Here a
// sweep advances iterations K+1 and K+2 at once: every scalar both of them
// need is a quadratic form in dot products of basis vectors that the
// PREVIOUS sweep could compute around its own outputs r_K, p_K (an s-step /
// communication-avoiding CG with s = 2, in the exact-expansion form of the
// single-reduction recurrence, without a stored basis):
//
//   z = D⁻¹r_K,  s = A p_K,  q = A z,  u = D⁻¹q,  v = D⁻¹s,  Au, Av
//   p₁ = z + β₁p,          A p₁ = q + β₁s
//   α₁ = (r,z)/(p₁,Ap₁),   r₁ = r − α₁Ap₁,   z₁ = z − α₁(u + β₁v)
//   (r₁,z₁) = (r,z) − 2α₁(z,Ap₁) + α₁²(Ap₁, D⁻¹Ap₁)   → β₂
//   p₂ = z₁ + β₂p₁ = (1+β₂)z + β₁β₂p − α₁u − α₁β₁v   → (p₂,Ap₂), ‖p₂‖² from
//   the A-Gram and the plain Gram of {z, p, u, v}          → α₂
//
// so the sweep reads r_K, p_K, w and writes r_{K+2}, p_{K+2}, w:
// 48 B per node per TWO iterations (24 B / iteration, against 40 for the
// single sweep with its deferred w update), and ONE 20-sum reduction per two
// iterations (half the cross-rank latency of the single sweep).  The stop
// test of both iterations is known before the sweep (|α₁|‖p₁‖, |α₂|‖p₂‖), so
// the iteration count and every terminal case keep the reference's exact
// semantics (stage2-mpi/poisson_mpi_decomp.cpp:400-457: breakdown before the
// update, stop after it); the sums are formed in a different order, which is
// the only numerical difference (the prototype and the device reproduce the
// golden counts: tests/test_gpu.py).
//
// Machine mapping (gfx950): the march of fused.hip with a 4-deep pipeline.
// Each wave64 strip loads 128 columns and outputs the middle 120 (lanes
// 2..61: the radius-4 dependence costs 2 lanes per side, all j-neighbours
// come from DPP lane shifts); rows march with five stages in flight
//   A  row t    p₁ = zc·D⁻¹r + β₁p                      (loads of row t)
//   B  row t−1  s₁ = Ap₁, r₁, z₁, p₂
//   C  row t−2  s₂ = Ap₂, r₂, z₂, v = D⁻¹s₂ → r₂, p₂, w += α₁p₁ + α₂p₂ stored
//   D  row t−3  q = Az₂, u = D⁻¹q
//   E  row t−4  Au, Av
// and each stage adds its row's share of the 20 sums.  Rotating row windows
// (period 2 or 3) live in registers; the loop is unrolled by 6 so every slot
// index is a compile-time constant.  Boundary-band rows (items with the band
// flag) evaluate their coefficients at each stage from the chord tables
// (division-free cset_rc; a few % of the row steps).
//
// Layout: fused.hip's (x[b] interleaves the r and p planes by row) with a
// 4-deep halo: local rows −3..nx+4 and columns −3..ny+4 hold data; buffer
// element 0 of a row is column −3.
#include <cstdlib>

#include "peer_sum.hpp"
#include "sstep.hpp"

#pragma clang fp contract(fast)

namespace pe {
namespace dev {

namespace {

constexpr int FSW2 = kFSW2;
#ifndef PE_S2_XD
#define PE_S2_XD 3
#endif
#ifndef PE_S2_WD
#define PE_S2_WD 3
#endif
constexpr int kS2XD = PE_S2_XD, kS2WD = PE_S2_WD;
constexpr int NS = kNS2;

// Scalars of the sweep covering iterations K+1, K+2 (K = st->iter) from the
// previous sweep's 20 unweighted sums R (a pure function of the state: every
// wave evaluates it and gets the same bits).  Sum layout (kNS2):
//   0 (r,z)  1 (z,q)  2 (z,s)  3 (p,s)  4 (q,u)  5 (u,s)  6 (s,v)  7 (u,Au)
//   8 (u,Av) 9 (v,Av) 10 (z,z) 11 (z,p) 12 (z,u) 13 (z,v) 14 (p,p) 15 (p,u)
//   16 (p,v) 17 (u,u) 18 (u,v) 19 (v,v)
struct Scal2 {
  bool first;
  long long K;
  double zc, g1, b1, den1, a1, d1, g2, b2, den2, a2, d2;
};

__device__ __forceinline__ double qform(const double (&c)[4], const double (&m)[4][4]) {
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s += c[i] * c[i] * m[i][i];
#pragma unroll
    for (int j = i + 1; j < 4; ++j) s += 2.0 * c[i] * c[j] * m[i][j];
  }
  return s;
}

__device__ __forceinline__ Scal2 sweep2_scalars(const KParams& k, const DevState* st, int par) {
  Scal2 c;
  c.first = st->started == 0;
  c.K = st->iter;
  c.zc = c.g1 = c.b1 = c.a1 = c.d1 = c.g2 = c.b2 = c.a2 = c.d2 = 0.0;
  c.den1 = c.den2 = 1.0;
  if (c.first) return c;
  const double hh = k.h1 * k.h2;
  const double* R = st->fs2[par ^ 1];
  c.zc = 1.0;
  c.g1 = R[0] * hh;
  c.b1 = c.K == 0 ? 0.0 : c.g1 / st->gprev;
  c.den1 = (R[1] + 2.0 * c.b1 * R[2] + c.b1 * c.b1 * R[3]) * hh;
  c.a1 = c.g1 / c.den1;
  const double pn1 = fmax(R[10] + 2.0 * c.b1 * R[11] + c.b1 * c.b1 * R[14], 0.0);
  c.d1 = k.weighted ? fabs(c.a1) * sqrt(pn1 * hh) : fabs(c.a1) * sqrt(pn1);
  c.g2 = (R[0] - 2.0 * c.a1 * (R[1] + c.b1 * R[2]) + c.a1 * c.a1 * (R[4] + 2.0 * c.b1 * R[5] + c.b1 * c.b1 * R[6])) * hh;
  c.b2 = c.g2 / c.g1;
  const double cf[4] = {1.0 + c.b2, c.b1 * c.b2, -c.a1, -c.a1 * c.b1};
  const double G[4][4] = {{R[1], R[2], R[4], R[5]}, {R[2], R[3], R[5], R[6]}, {R[4], R[5], R[7], R[8]},
                          {R[5], R[6], R[8], R[9]}};
  const double P[4][4] = {{R[10], R[11], R[12], R[13]}, {R[11], R[14], R[15], R[16]}, {R[12], R[15], R[17], R[18]},
                          {R[13], R[16], R[18], R[19]}};
  c.den2 = qform(cf, G) * hh;
  c.a2 = c.g2 / c.den2;
  const double pn2 = fmax(qform(cf, P), 0.0);
  c.d2 = k.weighted ? fabs(c.a2) * sqrt(pn2 * hh) : fabs(c.a2) * sqrt(pn2);
  return c;
}

// How the sweep ends the solve, if it does (a pure function of the scalars):
//   brk1  iteration K+1 breaks down (|den| < 1e-15 or non-finite scalars):
//         stop before its update (reference :413), w unchanged;
//   last1 iteration K+1 converges / hits the cap: w += α₁p₁ only;
//   brk2  iteration K+2 breaks down: w += α₁p₁ only (K+1 completed);
//   last2 iteration K+2 converges / hits the cap: the full sweep, then stop.
struct Term2 {
  bool brk1, bad1, last1, conv1, brk2, bad2, last2, conv2;
};
__device__ __forceinline__ Term2 sweep2_term(const KParams& k, const Scal2& c) {
  Term2 t{false, false, false, false, false, false, false, false};
  if (c.first) return t;
  const bool tiny1 = fabs(c.den1) < 1e-15;
  t.bad1 = !isfinite(c.g1) || !isfinite(c.den1) || (!tiny1 && !isfinite(c.d1));
  t.brk1 = t.bad1 || tiny1;
  if (t.brk1) return t;
  t.conv1 = k.check_tol && c.d1 < k.tol;
  t.last1 = t.conv1 || c.K + 1 >= k.max_iter;
  if (t.last1) return t;
  const bool tiny2 = fabs(c.den2) < 1e-15;
  t.bad2 = !isfinite(c.g2) || !isfinite(c.den2) || (!tiny2 && !isfinite(c.d2));
  t.brk2 = t.bad2 || tiny2;
  if (t.brk2) return t;
  t.conv2 = k.check_tol && c.d2 < k.tol;
  t.last2 = t.conv2 || c.K + 2 >= k.max_iter;
  return t;
}

// Terminal state of a sweep that stops before its own work (brk1 / last1 /
// brk2); one thread, after every wave of the grid has read the state.
__device__ __forceinline__ void sweep2_terminal(const KParams& k, DevState* st, const Scal2& c, const Term2& t) {
  if (t.brk1) {
    st->status = t.bad1 ? 4 : 2;
    st->iter = c.K + 1;
  } else {
    hist_put(k, c.K + 1, c.d1);
    st->last_diff = c.d1;
    st->alpha = c.a1;
    st->beta = c.b1;
    st->rz_cur = c.g1;
    st->gprev = c.g1;
    if (t.last1) {
      st->iter = c.K + 1;
      st->status = t.conv1 ? 1 : 3;
    } else {  // brk2
      st->iter = c.K + 2;
      st->status = t.bad2 ? 4 : 2;
    }
  }
  st->done = 1;
  st->wpend = 0;
}

// State update after a full sweep (one thread; sums t[] global).
__device__ __forceinline__ void sweep2_finalize(const KParams& k, DevState* st, int par, const Scal2& c,
                                                const Term2& tm, const double (&t)[NS]) {
#pragma unroll
  for (int n = 0; n < NS; ++n) st->fs2[par][n] = t[n];
  // fault hooks (PE_FAULT_INJECT): the sums of the sweep completing iteration K
  if (k.fault_iter > 0 && (c.K + 1 == k.fault_iter || c.K + 2 == k.fault_iter) && !c.first)
    st->fs2[par][1] = __builtin_nan("");
  if (k.fault_zero > 0 && (c.K + 1 == k.fault_zero || c.K + 2 == k.fault_zero) && !c.first)
    st->fs2[par][1] = st->fs2[par][2] = st->fs2[par][3] = 0.0;
  st->wpend = 0;
  st->wpar = par;
  if (c.first) {
    st->started = 1;
    return;
  }
  hist_put(k, c.K + 1, c.d1);
  hist_put(k, c.K + 2, c.d2);
  st->last_diff = c.d2;
  st->alpha = c.a2;
  st->beta = c.b2;
  st->rz_cur = c.g2;
  st->gprev = c.g2;
  st->iter = c.K + 2;
  if (tm.last2) {
    st->status = tm.conv2 ? 1 : 3;
    st->done = 1;
  }
}

// w += α₁ p₁ pointwise over the owned nodes (terminal paths last1 / brk2):
// p₁ = zc·D⁻¹r + β₁p from the input buffer, 1/D from the march's own
// coefficient path (cset_rc) so p₁ has the sweep's bits.
__device__ void w_add_p1(const KParams& k, const double* xin, const Scal2& c) {
  const int64_t n = k.nx * k.ny;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const double r = xin[li * k.pitch + lj], pold = xin[li * k.pitch + k.poff + lj];
    const int* rc = k.rowcls + (li + 1) * 4;
    const double* ctr = k.colT + (li + 1) * 4;
    const double* tv = k.rowT + (lj + 1) * 4;
    const double d = cset_rc(k, RowCls{rc[0], rc[1], rc[2], rc[3]}, CT{ctr[0], ctr[4], ctr[1], ctr[2]}, lj,
                             TV{tv[0], tv[1], tv[2], tv[6]}).d;
    const double p1 = c.zc * (r * d) + c.b1 * pold;
    double& w = k.w[li * k.wpitch + lj];
    w = w + c.a1 * p1;
  }
}

// The item march (one strip × rows ib..ie), accumulating this wave's sums.
// PUSH (row slabs over the P2P transport, KParams::push): output rows 1..4 /
// nx-3..nx are also stored into the x-neighbours' fine-grained receive
// buffers over xGMI (system-scope write-through stores, drained and released
// at the end of the item: delivered before this rank's cross-rank-sum flags),
// and the halo rows -3..0 / nx+1..nx+4 are read from this rank's receive
// buffer (system-scope loads) — fused.hip's halo push at depth 4.
// Sums are taken over the item's rows (uniform row tests) without per-term
// column masks: every sum has a factor among z, p, u, v, which are exactly 0
// at the global-boundary and padding columns (z, u, v masked there; p stays 0),
// and the lanes that do not own their columns (0, 1, 62, 63: the recomputed
// halo of the strip) are dropped once, at the end of the sweep.  (Blocks
// split across y — halo columns with real data — are not run by this kernel.)
template <bool BAND, bool PUSH>
__device__ __forceinline__ void march(const KParams& k, const Scal2& sc, int par, int s, int ib, int ie,
                                      WaveTV<6>& tvw, double (&acc)[NS]) {
  const int lane = threadIdx.x & 63;
  const int ny = int(k.ny);
  const int64_t pitch = k.pitch, poff = k.poff, wp = k.wpitch;
  const double* __restrict__ Xm = k.x[par ^ 1] - 3;  // row pointers at column -3
  double* __restrict__ Ym = k.x[par] - 3;
  double* __restrict__ Wm = k.w - 3;
  const int J = -3 + s * FSW2;
  const int c0 = J + 2 * lane;
  const int jl = 2 * lane;
  const unsigned off = unsigned(c0 + 3);
  const int64_t g0 = k.gj0 + c0;
  const bool lv0 = c0 <= ny + 4 && g0 >= 1 && g0 <= k.N - 1;
  const bool lv1 = c0 + 1 <= ny + 4 && g0 + 1 >= 1 && g0 + 1 <= k.N - 1;
  const bool inner = lane >= 2 && lane <= 61;
  const bool o0 = inner && c0 >= 1 && c0 <= ny;
  const bool o1 = inner && c0 + 1 >= 1 && c0 + 1 <= ny;
  const double a1 = sc.a1, b1 = sc.b1, a2 = sc.a2, b2 = sc.b2, zc = sc.zc;

  const int t0 = ib - 4;
  // Row classes / column tables of rows segbase .. segbase+63 (one per lane),
  // reloaded every ~54 rows on tall items (stage rows t-4 .. t and the
  // column-table row t+1 stay inside the window).
  RowCtx rx;
  auto load_seg = [&](int base) { load_rows<BAND>(k, rx, tvw, base, ie + 5, J); };
  if (BAND) load_strip_tables(k, tvw, c0);  // the strip's row-table entries, once per band item
  load_seg(t0);
  auto interior = [&](int q) {  // global interior row
    const int64_t gr = k.gi0 + q;
    return gr >= 1 && gr <= k.M - 1;
  };
  const int nx = int(k.nx);
  // receive buffer of the parity this sweep reads: [side][4 rows], rows from column -3
  const double* hrd = PUSH ? k.hrecv + int64_t(par ^ 1) * 8 * pitch : nullptr;
  auto ldx = [&](int t, unsigned o) -> double2 {
    if constexpr (PUSH) {
      if ((t < 1 && k.has[LEFT]) || (t > nx && k.has[RIGHT])) {
        const double* h = hrd + int64_t(t < 1 ? t + 3 : t - nx + 3) * pitch + o;
        return dd(__hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                  __hip_atomic_load(h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      }
    }
    return ld2(Xm + int64_t(t) * pitch + o);
  };
  bool pushed = false;
  auto push_row = [&](int q, const double2& r2, const double2& p2) {
    auto put = [&](double* base, int slot) {
      double* d = base + int64_t(slot) * pitch + off;
      if (o0) {
        __hip_atomic_store(d, r2.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d + poff, p2.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (o1) {
        __hip_atomic_store(d + 1, r2.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d + 1 + poff, p2.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      pushed = true;
    };
    // rows 1..4 → the LEFT neighbour's rows nx'+1..nx'+4; nx-3..nx → the RIGHT one's -3..0
    if (q <= 4 && k.hpush_lo[par] != nullptr) put(k.hpush_lo[par], q - 1);
    if (q >= nx - 3 && k.hpush_hi[par] != nullptr) put(k.hpush_hi[par], q - (nx - 3));
  };

  // prefetch ring (3 rows): x rows t, t+1, t+2; w rows t-2, t-1, t
  const int tmax = ie + 4;
  // rows of loads in flight: x (r, p) XD, w WD (each 2 or 3: divides the unroll)
  constexpr int XD = kS2XD, WD = kS2WD;
  double2 RQ[XD], PQ[XD], WQ[WD];
#pragma unroll
  for (int q = 0; q < XD; ++q) {
    const int t = min(t0 + q, tmax);
    RQ[q] = ldx(t, off);
    PQ[q] = ldx(t, poff + off);
  }
#pragma unroll
  for (int q = 0; q < WD; ++q) WQ[q] = ldnt(Wm + int64_t(min(max(t0 - 2 + q, ib), ie)) * wp + off);
  double2 P1[3], RI[2], R1[2], P2[3], Z2[3], S2[2], V[3], U[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) P1[q] = P2[q] = Z2[q] = V[q] = U[q] = dd(0.0, 0.0);
#pragma unroll
  for (int q = 0; q < 2; ++q) RI[q] = R1[q] = S2[q] = dd(0.0, 0.0);
  double (&sv)[NS] = acc;  // the wave's running sums

  const int nsteps = ie + 4 - t0 + 1;
  for (int g = 0; 6 * g < nsteps; ++g) {
    if (t0 + 6 * g + 6 - rx.segbase > 63) load_seg(t0 + 6 * g - 4);  // tall items: next row window
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      const int n = 6 * g + jj;
      if (n >= nsteps) break;
      const int t = t0 + n;
      // slots (compile-time): m3[d] = (n - d) mod 3, m2[d] = (n - d) mod 2
      const int s0 = jj % 3, s1 = (jj + 2) % 3, s2 = (jj + 1) % 3;  // rows t, t-1, t-2 (mod 3): t-3 ≡ t
      const int e0 = jj & 1, e1 = (jj + 1) & 1;                     // rows t, t-1 (mod 2): t-2 ≡ t
      const int r0 = jj, r1s = (jj + 5) % 6, r2s = (jj + 4) % 6;    // band ring slots (mod 6) of rows t .. t-4
      const int r3s = (jj + 3) % 6, r4s = (jj + 2) % 6;
      // ---- A: row t ----
      const int xs = jj % XD, ws = jj % WD;
      const double2 rin = RQ[xs], pin = PQ[xs], wrow = WQ[ws];
      {
        const int tn = min(t + XD, tmax);
        RQ[xs] = ldx(tn, off);
        PQ[xs] = ldx(tn, poff + off);
        WQ[ws] = ldnt(Wm + int64_t(min(max(t - 2 + WD, ib), ie)) * wp + off);
      }
      {
        const double2 d = BAND ? enter_band(k, rx, tvw, t, c0, jl, r0) : dinv_plain(k, rx, t, c0);
        const bool ri = interior(t);
        const double z0 = (ri && lv0) ? rin.x * d.x : 0.0, z1 = (ri && lv1) ? rin.y * d.y : 0.0;
        P1[s0] = dd(zc * z0 + b1 * pin.x, zc * z1 + b1 * pin.y);
        RI[e0] = rin;
      }
      // ---- B: row t-1 ----
      {
        double2 d;
        const double2 s1v = apply_row<BAND>(k, rx, tvw, t - 1, c0, jl, r1s, r0, P1[s2], P1[s1], P1[s0], d);
        const double2 ri = RI[e1];
        const double2 r1 = dd(ri.x - a1 * s1v.x, ri.y - a1 * s1v.y);
        const bool rr = interior(t - 1);
        const double z0 = (rr && lv0) ? r1.x * d.x : 0.0, z1 = (rr && lv1) ? r1.y * d.y : 0.0;
        const double2 p1 = P1[s1];
        R1[e1] = r1;
        P2[s1] = dd(zc * z0 + b2 * p1.x, zc * z1 + b2 * p1.y);
      }
      // ---- C: row t-2 (outputs) ----
      {
        const int q = t - 2;
        double2 d;
        const double2 s2v = apply_row<BAND>(k, rx, tvw, q, c0, jl, r2s, r1s, P2[s0], P2[s2], P2[s1], d);
        const double2 r1 = R1[e0];
        const double2 r2 = dd(r1.x - a2 * s2v.x, r1.y - a2 * s2v.y);
        const bool rr = interior(q);
        const double2 z2 = dd((rr && lv0) ? r2.x * d.x : 0.0, (rr && lv1) ? r2.y * d.y : 0.0);
        Z2[s2] = z2;
        S2[e0] = s2v;
        const double2 p2 = P2[s2];
        if (q >= ib && q <= ie) {
          const double2 p1 = P1[s2];
          const double2 wv = dd(wrow.x + a1 * p1.x + a2 * p2.x, wrow.y + a1 * p1.y + a2 * p2.y);
          double* yr = Ym + int64_t(q) * pitch + off;
          double* wd = Wm + int64_t(q) * wp + off;
          if (o0 && o1) {
            st2nt(yr, r2);
            st2nt(yr + poff, p2);
            st2nt(wd, wv);
          } else if (o0) {
            yr[0] = r2.x;
            yr[poff] = p2.x;
            wd[0] = wv.x;
          }
          if constexpr (PUSH) push_row(q, r2, p2);
          sv[0] += r2.x * z2.x + r2.y * z2.y;            // (r,z)
          sv[2] += z2.x * s2v.x + z2.y * s2v.y;          // (z,s)
          sv[3] += p2.x * s2v.x + p2.y * s2v.y;          // (p,s)
          sv[10] += z2.x * z2.x + z2.y * z2.y;           // (z,z)
          sv[11] += z2.x * p2.x + z2.y * p2.y;           // (z,p)
          sv[14] += p2.x * p2.x + p2.y * p2.y;           // (p,p)
        }
      }
      // ---- D: row t-3 ----
      {
        const int q = t - 3;
        double2 d;
        const double2 qv = apply_row<BAND>(k, rx, tvw, q, c0, jl, r3s, r2s, Z2[s1], Z2[s0], Z2[s2], d);
        const bool rr = interior(q);
        const double2 sr = S2[e1];
        const double2 u = dd((rr && lv0) ? qv.x * d.x : 0.0, (rr && lv1) ? qv.y * d.y : 0.0);
        const double2 v = dd((rr && lv0) ? sr.x * d.x : 0.0, (rr && lv1) ? sr.y * d.y : 0.0);
        U[s0] = u;
        V[s0] = v;
        if (q >= ib && q <= ie) {
          const double2 z = Z2[s0], p = P2[s0];
          sv[1] += z.x * qv.x + z.y * qv.y;              // (z,q)
          sv[4] += qv.x * u.x + qv.y * u.y;              // (q,u)
          sv[5] += u.x * sr.x + u.y * sr.y;              // (u,s)
          sv[6] += sr.x * v.x + sr.y * v.y;              // (s,v)
          sv[12] += z.x * u.x + z.y * u.y;               // (z,u)
          sv[13] += z.x * v.x + z.y * v.y;               // (z,v)
          sv[15] += p.x * u.x + p.y * u.y;               // (p,u)
          sv[16] += p.x * v.x + p.y * v.y;               // (p,v)
          sv[17] += u.x * u.x + u.y * u.y;               // (u,u)
          sv[18] += u.x * v.x + u.y * v.y;               // (u,v)
          sv[19] += v.x * v.x + v.y * v.y;               // (v,v)
        }
      }
      // ---- E: row t-4 ----
      {
        const int q = t - 4;
        if (q >= ib && q <= ie) {
          double2 d;
          const double2 au = apply_row<BAND>(k, rx, tvw, q, c0, jl, r4s, r3s, U[s2], U[s1], U[s0], d);
          const double2 av = apply_row<BAND>(k, rx, tvw, q, c0, jl, r4s, r3s, V[s2], V[s1], V[s0], d);
          const double2 u = U[s1], v = V[s1];
          sv[7] += u.x * au.x + u.y * au.y;              // (u,Au)
          sv[8] += u.x * av.x + u.y * av.y;              // (u,Av)
          sv[9] += v.x * av.x + v.y * av.y;              // (v,Av)
        }
      }
    }
  }
  if constexpr (PUSH) {
    if (pushed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (system-scope atomic stores: fused3.hip march3)
  }
}

template <bool PUSH>
__global__ __launch_bounds__(TJ) __attribute__((amdgpu_waves_per_eu(2))) void kS2(KParams k, int par) {
  DevState* st = k.st;
  const int done = st->done;
  const Scal2 sc = sweep2_scalars(k, st, par);
  const Term2 tm = sweep2_term(k, sc);
  __shared__ double sm[4 * NS];
  __shared__ int sflag;
  __shared__ WaveTV<6> tvs[kWPB];
  const int lane = int(threadIdx.x & 63);
  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  if (done) return;
  if (tm.brk1 || tm.last1 || tm.brk2) {
    if (!tm.brk1) w_add_p1(k, k.x[par ^ 1], sc);
    if (arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
      sweep2_terminal(k, st, sc, tm);
      __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  double acc[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  {  // band ring: defined contents (the never-written column 128 of b0 and the
     // slots garbage pipeline-fill rows read stay finite)
    WaveTV<6>& tv = tvs[wid];
    for (int i = lane; i < 6 * 128; i += 64) (&tv.a0r[0][0])[i] = 0.0;
    for (int i = lane; i < 6 * 130; i += 64) (&tv.b0r[0][0])[i] = 0.0;
  }
  const int W = k.lwaves;
  // (waves past the layout's W — a grid with reserved blocks — have no positions)
  for (int pos = int(blockIdx.x) * kWPB + wid < W ? int(blockIdx.x) * kWPB + wid : k.nslots; pos < k.nslots; pos += W) {
    const int2 e = cload_i2(k.ilist + pos);
    const int rows = e.y >> 20;
    if (rows == 0) continue;  // empty position of the static layout
    const int s = e.y & 0xFFFFF, ib = e.x & kRowMask;
    const int ie = min(ib + rows - 1, int(k.nx));
    if (e.x & kBandBit) march<true, PUSH>(k, sc, par, s, ib, ie, tvs[wid], acc);
    else march<false, PUSH>(k, sc, par, s, ib, ie, tvs[wid], acc);
  }
  if (lane < 2 || lane > 61)  // strip halo lanes: recomputed copies of the neighbouring strips' columns
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  if (publish_last_nm<NS>(k.partial, acc, &st->ticket[0], &sflag, sm)) {  // (kcommon.hpp: n-major partials)
    double t[NS];
    reduce_partials_nm<NS>(k.partial, t, sm);
    __shared__ double xv[NS + 1];
    __shared__ unsigned long long sseq;
    __shared__ int sok;
    if (k.xr.peers) {  // cross-rank sum of the 20 sums inside the sweep (P2P transport)
      if (threadIdx.x == 0) {
#pragma unroll
        for (int n = 0; n < NS; ++n) xv[n] = t[n];
        if (k.slow_ticks > 0) {  // PE_FAULT_INJECT=slow@rank (test hook): idle before the cross-rank sum
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < k.slow_ticks) __builtin_amdgcn_s_sleep(2);
        }
      }
      peer_sum_block(k.xr, xv, NS, &sseq, &sok);
      if (threadIdx.x == 0)
#pragma unroll
        for (int n = 0; n < NS; ++n) t[n] = xv[n];
    }
    if (threadIdx.x == 0) {
      sweep2_finalize(k, st, par, sc, tm, t);
      __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

void launch_S2(const KParams& k, int par, hipStream_t s) {
  if (k.push) hipLaunchKernelGGL(kS2<true>, dim3(unsigned(k.nblocks)), dim3(TJ), 0, s, k, par);
  else hipLaunchKernelGGL(kS2<false>, dim3(unsigned(k.nblocks)), dim3(TJ), 0, s, k, par);
}

int resident_blocks_S2() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kS2<false>, TJ, 0) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  return n;
}

}  // namespace dev
}  // namespace pe
