// Three-step single sweep: THREE Jacobi-PCG iterations per pass over memory.
//
// fused2.hip advances two iterations per pass from sums the previous pass
// formed around its outputs; this kernel takes the s-step recurrence one
// step further (s = 3).  With M = D⁻¹A (self-adjoint in the D inner
// product), every scalar of iterations K+1..K+3 is a quadratic form in the
// D-moments of z = D⁻¹r_K and p = p_K,
//
//   μ_n(x, y) = (x, D Mⁿ y),   n = 0..5,
//
// since r_{K+i-1} = D z_{K+i-1} and p_{K+i} are polynomials of degree ≤ 2 in
// M applied to z and p (tools/sstep_proto.py; the prototype and the device
// reproduce every golden iteration count up to 8192²:
// profiles/r3_sstep3_numerics.txt).  Each moment is ONE dot product of
// vectors the sweep forms anyway:
//
//   q = Az, u = D⁻¹q, v = D⁻¹s (s = Ap), Au, Av, ũ = D⁻¹Au, ṽ = D⁻¹Av, Aũ, Aṽ
//   zz: (r,z) (z,q) (q,u) (u,Au) (Au,ũ) (ũ,Aũ)      — sums 0..5
//   zp:       (z,s) (q,v) (u,Av) (Au,ṽ) (ũ,Aṽ)      — sums 6..10
//   pp:       (p,s) (s,v) (v,Av) (Av,ṽ) (ṽ,Aṽ)      — sums 11..15
//
// (μ_0 of zp / pp never enters: z_{K+i} has p-components of degree ≥ 1.)
// The stop test of iteration K+i, |α_i|‖p_i‖, uses ‖p_i‖² summed by the
// sweep that forms p_i (sums 16..18) — "late": a sweep that converges on its
// first or second iteration has already added the later α_j p_j to w, and
// the next launch subtracts them again (fix-up mode: the same march over the
// same inputs with the saved scalars, w -= α_j p_j only).  Breakdown (|den| <
// 1e-15) and the iteration cap are known before the sweep: the sweep applies
// only the iterations before them (an identity step is zc = 0, β = 1, α = 0).
// So the iteration count and every terminal case keep the reference's
// semantics (stage2-mpi/poisson_mpi_decomp.cpp:400-457); the moments are
// summed in a different order, which is the only numerical difference.
//
// Traffic: r_K, p_K, w in, r_{K+3}, p_{K+3}, w out: 48 B per node per THREE
// iterations (16 B / iteration, against 24 two-step and 40 single sweep) and
// one 19-sum reduction per three iterations.
//
// Machine mapping (gfx950): fused2.hip's march with a 6-deep pipeline.  Each
// wave64 strip loads 128 columns and outputs the middle 116 (lanes 3..60:
// radius-6 dependence); rows march with seven stages in flight
//   A  row t    p₁ = zc₁D⁻¹r + β₁p                          (loads of row t)
//   B  row t−1  s₁ = Ap₁, r₁, z₁, p₂                         ‖p₁‖²
//   C  row t−2  s₂ = Ap₂, r₂, z₂, p₃, w += Σ α_i p_i stored  ‖p₂‖²
//   D  row t−3  s = Ap₃, r₃, z = D⁻¹r₃ → r₃, p₃ stored       (r,z) (z,s) (p,s) ‖p₃‖²
//   E  row t−4  q = Az, u, v                                 (z,q) (q,u) (q,v) (s,v)
//   F  row t−5  Au, Av, ũ, ṽ                                 (u,Au) (u,Av) (v,Av) (Au,ũ) (Au,ṽ) (Av,ṽ)
//   G  row t−6  Aũ, Aṽ                                        (ũ,Aũ) (ũ,Aṽ) (ṽ,Aṽ)
// with register rings of period 2 / 3 (unroll 6) and, for band items, a
// 7-row LDS ring of face coefficients (runtime slot: row − t0 mod 7).
//
// Layout: fused.hip's (x[b] interleaves the r and p planes by row) with a
// 6-deep halo: local rows −5..nx+6 and columns −5..ny+6 hold data; buffer
// element 0 of a row is column −5.
#include <cstdlib>

#include "peer_sum.hpp"
#include "sstep.hpp"

#pragma clang fp contract(fast)

namespace pe {
namespace dev {

namespace {

constexpr int H3 = 6;
constexpr int FSW3 = kFSW3;
static_assert(FSW3 == 128 - 2 * H3, "three-step strip: 128 loaded columns, H3 halo columns per side");
#ifndef PE_S3_XD
#define PE_S3_XD 3
#endif
#ifndef PE_S3_WD
#define PE_S3_WD 3
#endif
constexpr int kS3XD = PE_S3_XD, kS3WD = PE_S3_WD;
constexpr int NS = kNS3;
constexpr int kRing3 = 7;  // band face ring: rows t-6 .. t
using WaveTV3 = WaveTV<kRing3>;

// Scalars of a sweep (iterations K+1 .. K+m).  Iteration i applies
//   p_i = zc_i·z_{i-1} + β_i p_{i-1},  r_i = r_{i-1} − α_i A p_i
// and w += Σ cw_i p_i (cw = α; fix-up: −α_j of the iterations past the stop).
struct Coef3 {
  double zc[3], a[3], b[3], cw[3];
};

struct Scal3 {
  bool first;
  long long K;
  int m;    // iterations this sweep applies (0..3)
  int brk;  // 1..3: that iteration breaks down before its update (it follows the m applied ones); 0 none
  bool bad; // the breakdown is a non-finite scalar
  Coef3 c;
  double g[3];  // (r, z) before each applied iteration, h-weighted
};

// Quadratic form Σ_{a,b} x_a x_b μ_{a+b+sh} of the coefficient vector
// x = Σ_a xz_a M^a z + xp_a M^a p (sh = 0: D-form, sh = 1: A-form).
__device__ __forceinline__ double mform(const double (&xz)[3], const double (&xp)[3], const double (&mzz)[6],
                                        const double (&mzp)[6], const double (&mpp)[6], int sh) {
  double s = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int n = a + b + sh;
      s += xz[a] * (xz[b] * mzz[n] + 2.0 * xp[b] * mzp[n]) + xp[a] * xp[b] * mpp[n];
    }
  return s;
}

// From the previous sweep's 19 unweighted sums (a pure function of the state:
// every wave evaluates it and gets the same bits).
__device__ __forceinline__ Scal3 sweep3_scalars(const KParams& k, const DevState* st, int par) {
  Scal3 c;
  c.first = st->started == 0;
  c.K = st->iter;
  c.m = 0;
  c.brk = 0;
  c.bad = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    c.c.zc[i] = 0.0;
    c.c.a[i] = 0.0;
    c.c.b[i] = 1.0;
    c.c.cw[i] = 0.0;
    c.g[i] = 0.0;
  }
  if (c.first) return c;
  const double hh = k.h1 * k.h2;
  const double* R = st->fs2[par ^ 1];
  const double mzz[6] = {R[0], R[1], R[2], R[3], R[4], R[5]};
  const double mzp[6] = {0.0, R[6], R[7], R[8], R[9], R[10]};
  const double mpp[6] = {0.0, R[11], R[12], R[13], R[14], R[15]};
  long long lim = k.max_iter - c.K;
  if (lim > 3) lim = 3;
  if (k.mlimit > 0 && lim > k.mlimit) lim = k.mlimit;
  double zz[3] = {1.0, 0.0, 0.0}, zp[3] = {0.0, 0.0, 0.0};  // z_{i-1}
  double pz[3] = {0.0, 0.0, 0.0}, pp[3] = {1.0, 0.0, 0.0};  // p_{i-1}
  double g = mform(zz, zp, mzz, mzp, mpp, 0) * hh;
  double gprev = st->gprev;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i >= lim) break;
    const double beta = c.K + i == 0 ? 0.0 : g / gprev;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      pz[q] = zz[q] + beta * pz[q];
      pp[q] = zp[q] + beta * pp[q];
    }
    const double den = mform(pz, pp, mzz, mzp, mpp, 1) * hh;
    const bool tiny = fabs(den) < 1e-15;
    const bool bad = !isfinite(g) || !isfinite(den);
    if (tiny || bad) {
      c.brk = i + 1;
      c.bad = bad;
      break;
    }
    const double alpha = g / den;
    c.c.zc[i] = 1.0;
    c.c.a[i] = alpha;
    c.c.b[i] = beta;
    c.c.cw[i] = alpha;
    c.g[i] = g;
    c.m = i + 1;
    gprev = g;
    if (i + 1 < lim) {  // z_i = z_{i-1} − α M p_i
      zz[2] -= alpha * pz[1];
      zz[1] -= alpha * pz[0];
      zp[2] -= alpha * pp[1];
      zp[1] -= alpha * pp[0];
      g = mform(zz, zp, mzz, mzp, mpp, 0) * hh;
    }
  }
  return c;
}

// Iteration K+1 breaks down before its update: stop, w unchanged (one
// thread, after every wave of the grid has read the state).
__device__ __forceinline__ void sweep3_terminal(DevState* st, const Scal3& c) {
  st->status = c.bad ? 4 : 2;
  st->iter = c.K + 1;
  st->done = 1;
  st->wpend = 0;
}

// State update after a full sweep (one thread; sums t[] global): the late
// stop tests of the m applied iterations, then breakdown / cap.
__device__ __forceinline__ void sweep3_finalize(const KParams& k, DevState* st, int par, const Scal3& c,
                                                const double (&t)[NS]) {
#pragma unroll
  for (int n = 0; n < NS; ++n) st->fs2[par][n] = t[n];
  // fault hooks (PE_FAULT_INJECT): the sums of the sweep completing iteration F
  if (!c.first && k.fault_iter > c.K && k.fault_iter <= c.K + c.m) st->fs2[par][1] = __builtin_nan("");
  if (!c.first && k.fault_zero > c.K && k.fault_zero <= c.K + c.m)
    st->fs2[par][1] = st->fs2[par][6] = st->fs2[par][11] = 0.0;
  st->wpend = 0;
  st->wpar = par;
  if (c.first) {
    st->started = 1;
    return;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st->sc3[i] = c.c.zc[i];
    st->sc3[3 + i] = c.c.a[i];
    st->sc3[6 + i] = c.c.b[i];
    st->sc3[9 + i] = 0.0;
  }
  const double hh = k.h1 * k.h2;
  int stop = 0, status = 0;
  for (int i = 0; i < c.m; ++i) {
    const double n2 = fmax(t[16 + i], 0.0);
    const double d = k.weighted ? fabs(c.c.a[i]) * sqrt(n2 * hh) : fabs(c.c.a[i]) * sqrt(n2);
    hist_put(k, c.K + i + 1, d);
    st->last_diff = d;
    st->alpha = c.c.a[i];
    st->beta = c.c.b[i];
    st->rz_cur = c.g[i];
    st->gprev = c.g[i];
    st->iter = c.K + i + 1;
    if (!isfinite(d)) {
      status = 4;
      stop = i + 1;
      break;
    }
    if (k.check_tol && d < k.tol) {
      status = 1;
      stop = i + 1;
      break;
    }
  }
  if (stop == 0) {
    if (c.brk) {
      st->iter = c.K + c.brk;
      status = c.bad ? 4 : 2;
    } else if (c.K + c.m >= k.max_iter) {
      status = 3;
    }
  } else if (stop < c.m && status == 1) {  // w holds the later iterations' terms: the next launch subtracts them
    for (int j = stop; j < c.m; ++j) st->sc3[9 + j] = -c.c.a[j];
    st->fixpend = 1;
  }
  if (status) {
    st->status = status;
    st->done = 1;
  }
}

// The item march (one strip × rows ib..ie), accumulating this wave's sums.
// FIX (fix-up launch): same march over the same inputs, w only.
// PUSH (row slabs over the P2P transport): output rows 1..6 / nx-5..nx are
// also stored into the x-neighbours' fine-grained receive buffers over xGMI
// (system-scope write-through stores, drained and released at the end of the
// item), and the halo rows -5..0 / nx+1..nx+6 are read from this rank's
// receive buffer (system-scope loads) — fused2.hip's halo push at depth 6.
// Sums are taken over the item's rows without per-term column masks: every
// sum has a factor among z, p, u, v, ũ, ṽ, which are exactly 0 at the
// global-boundary and padding columns, and the lanes that do not own their
// columns (0..2, 61..63) are dropped once, at the end of the sweep.
template <bool BAND, bool PUSH>
__device__ __forceinline__ void march3(const KParams& k, const Coef3& cf, bool fix, int par, int s, int ib, int ie,
                                       WaveTV3& tvw, double (&sv)[NS]) {
  const int lane = threadIdx.x & 63;
  const int ny = int(k.ny);
  const int64_t pitch = k.pitch, poff = k.poff, wp = k.wpitch;
  const double* __restrict__ Xm = k.x[par ^ 1] - (H3 - 1);  // row pointers at column -5
  double* __restrict__ Ym = k.x[par] - (H3 - 1);
  double* __restrict__ Wm = k.w - (H3 - 1);
  const int J = -(H3 - 1) + s * FSW3;
  const int c0 = J + 2 * lane;
  const int jl = 2 * lane;
  const unsigned off = unsigned(c0 + H3 - 1);
  const int64_t g0 = k.gj0 + c0;
  const bool lv0 = c0 <= ny + H3 && g0 >= 1 && g0 <= k.N - 1;
  const bool lv1 = c0 + 1 <= ny + H3 && g0 + 1 >= 1 && g0 + 1 <= k.N - 1;
  const bool inner = lane >= 3 && lane <= 60;
  const bool o0 = inner && c0 >= 1 && c0 <= ny;
  const bool o1 = inner && c0 + 1 >= 1 && c0 + 1 <= ny;
  const double zc1 = cf.zc[0], zc2 = cf.zc[1], zc3 = cf.zc[2];
  const double a1 = cf.a[0], a2 = cf.a[1], a3 = cf.a[2];
  const double b1 = cf.b[0], b2 = cf.b[1], b3 = cf.b[2];
  const double w1 = cf.cw[0], w2 = cf.cw[1], w3 = cf.cw[2];

  const int t0 = ib - H3;
  // Row classes / column tables of a 64-row window, reloaded every ~58 rows
  // on tall items (stage rows t-6 .. t and the column-table row t+1 inside).
  RowCtx rx;
  auto load_seg = [&](int base) { load_rows<BAND>(k, rx, tvw, base, ie + H3 + 1, J); };
  if (BAND) load_strip_tables(k, tvw, c0);
  load_seg(t0);
  auto interior = [&](int q) {  // global interior row
    const int64_t gr = k.gi0 + q;
    return gr >= 1 && gr <= k.M - 1;
  };
  const int nx = int(k.nx);
  // receive buffer of the parity this sweep reads: [side][6 rows], rows from column -5
  const double* hrd = PUSH ? k.hrecv + int64_t(par ^ 1) * 2 * H3 * pitch : nullptr;
  auto ldx = [&](int t, unsigned o) -> double2 {
    if constexpr (PUSH) {
      if ((t < 1 && k.has[LEFT]) || (t > nx && k.has[RIGHT])) {
        const double* h = hrd + int64_t(t < 1 ? t + H3 - 1 : t - nx + H3 - 1) * pitch + o;
        return dd(__hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                  __hip_atomic_load(h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      }
    }
    return ld2(Xm + int64_t(t) * pitch + o);
  };
  bool pushed = false;
  auto push_row = [&](int q, const double2& r3, const double2& p3) {
    auto put = [&](double* base, int slot) {
      double* d = base + int64_t(slot) * pitch + off;
      if (o0) {
        __hip_atomic_store(d, r3.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d + poff, p3.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (o1) {
        __hip_atomic_store(d + 1, r3.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d + 1 + poff, p3.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      pushed = true;
    };
    // rows 1..6 → the LEFT neighbour's rows nx'+1..nx'+6; nx-5..nx → the RIGHT one's -5..0
    if (q <= H3 && k.hpush_lo[par] != nullptr) put(k.hpush_lo[par], q - 1);
    if (q >= nx - H3 + 1 && k.hpush_hi[par] != nullptr) put(k.hpush_hi[par], q - (nx - H3 + 1));
  };

  const int tmax = ie + H3;
  // rows of loads in flight: x (r, p) XD, w WD (each 2 or 3: divides the unroll);
  // w is consumed at stage C (row t-2)
  constexpr int XD = kS3XD, WD = kS3WD;
  double2 RQ[XD], PQ[XD], WQ[WD];
#pragma unroll
  for (int q = 0; q < XD; ++q) {
    const int t = min(t0 + q, tmax);
    RQ[q] = ldx(t, off);
    PQ[q] = ldx(t, poff + off);
  }
#pragma unroll
  for (int q = 0; q < WD; ++q) WQ[q] = ldnt(Wm + int64_t(min(max(t0 - 2 + q, ib), ie)) * wp + off);
  double2 P1[3], RI[2], R1[2], P2[3], R2[2], P3[3], Z[3], S[2], U[3], V[3], UU[3], VV[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) P1[q] = P2[q] = P3[q] = Z[q] = U[q] = V[q] = UU[q] = VV[q] = dd(0.0, 0.0);
#pragma unroll
  for (int q = 0; q < 2; ++q) RI[q] = R1[q] = R2[q] = S[q] = dd(0.0, 0.0);

  const int nsteps = ie + H3 - t0 + 1;
  int bs = 0;  // band ring slot of row t: (t - t0) mod 7
  for (int g = 0; 6 * g < nsteps; ++g) {
    if (t0 + 6 * g + 6 - rx.segbase > 63) load_seg(t0 + 6 * g - H3);  // tall items: next row window
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      const int n = 6 * g + jj;
      if (n >= nsteps) break;
      const int t = t0 + n;
      // register ring slots (compile-time): row t-d ↦ (jj - d) mod 3 / mod 2
      const int m0 = jj % 3, m1 = (jj + 2) % 3, m2 = (jj + 1) % 3;  // rows t, t-1, t-2 (t-3 ≡ t)
      const int e0 = jj & 1, e1 = (jj + 1) & 1;                      // rows t, t-1 (t-2 ≡ t)
      // band ring slots (runtime, mod 7) of rows t .. t-6
      int bsl[7];
#pragma unroll
      for (int d = 0; d < 7; ++d) bsl[d] = bs >= d ? bs - d : bs - d + kRing3;
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
        const double2 d = BAND ? enter_band(k, rx, tvw, t, c0, jl, bsl[0]) : dinv_plain(k, rx, t, c0);
        const bool ri = interior(t);
        const double z0 = (ri && lv0) ? rin.x * d.x : 0.0, z1 = (ri && lv1) ? rin.y * d.y : 0.0;
        P1[m0] = dd(zc1 * z0 + b1 * pin.x, zc1 * z1 + b1 * pin.y);
        RI[e0] = rin;
      }
      // ---- B: row t-1 ----
      {
        const int q = t - 1;
        double2 d;
        const double2 s1 = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[1], bsl[0], P1[m2], P1[m1], P1[m0], d);
        const double2 ri = RI[e1];
        const double2 r1 = dd(ri.x - a1 * s1.x, ri.y - a1 * s1.y);
        const bool rr = interior(q);
        const double z0 = (rr && lv0) ? r1.x * d.x : 0.0, z1 = (rr && lv1) ? r1.y * d.y : 0.0;
        const double2 p1 = P1[m1];
        R1[e1] = r1;
        P2[m1] = dd(zc2 * z0 + b2 * p1.x, zc2 * z1 + b2 * p1.y);
        if (q >= ib && q <= ie) sv[16] += dot2(p1, p1);
      }
      // ---- C: row t-2 (w) ----
      {
        const int q = t - 2;
        double2 d;
        const double2 s2 = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[2], bsl[1], P2[m0], P2[m2], P2[m1], d);
        const double2 r1 = R1[e0];
        const double2 r2 = dd(r1.x - a2 * s2.x, r1.y - a2 * s2.y);
        const bool rr = interior(q);
        const double z0 = (rr && lv0) ? r2.x * d.x : 0.0, z1 = (rr && lv1) ? r2.y * d.y : 0.0;
        const double2 p2 = P2[m2];
        R2[e0] = r2;
        const double2 p3 = dd(zc3 * z0 + b3 * p2.x, zc3 * z1 + b3 * p2.y);
        P3[m2] = p3;
        if (q >= ib && q <= ie) {
          const double2 p1 = P1[m2];
          const double2 wv = dd(wrow.x + w1 * p1.x + w2 * p2.x + w3 * p3.x, wrow.y + w1 * p1.y + w2 * p2.y + w3 * p3.y);
          double* wd = Wm + int64_t(q) * wp + off;
          if (o0 && o1) st2nt(wd, wv);
          else if (o0) wd[0] = wv.x;
          sv[17] += dot2(p2, p2);
        }
      }
      // ---- D: row t-3 (r, p outputs) ----
      {
        const int q = t - 3;
        double2 d;
        const double2 s3 = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[3], bsl[2], P3[m1], P3[m0], P3[m2], d);
        const double2 r2 = R2[e1];
        const double2 r3 = dd(r2.x - a3 * s3.x, r2.y - a3 * s3.y);
        const bool rr = interior(q);
        const double2 z = dd((rr && lv0) ? r3.x * d.x : 0.0, (rr && lv1) ? r3.y * d.y : 0.0);
        Z[m0] = z;
        S[e1] = s3;
        if (q >= ib && q <= ie) {
          const double2 p3 = P3[m0];
          if (!fix) {
            double* yr = Ym + int64_t(q) * pitch + off;
            if (o0 && o1) {
              st2nt(yr, r3);
              st2nt(yr + poff, p3);
            } else if (o0) {
              yr[0] = r3.x;
              yr[poff] = p3.x;
            }
            if constexpr (PUSH) push_row(q, r3, p3);
          }
          sv[0] += dot2(r3, z);   // (r,z)
          sv[6] += dot2(z, s3);   // (z,s)
          sv[11] += dot2(p3, s3); // (p,s)
          sv[18] += dot2(p3, p3); // ‖p₃‖²
        }
      }
      // ---- E: row t-4 ----
      {
        const int q = t - 4;
        double2 d;
        const double2 qv = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[4], bsl[3], Z[m2], Z[m1], Z[m0], d);
        const bool rr = interior(q);
        const double2 sr = S[e0];
        const double2 u = dd((rr && lv0) ? qv.x * d.x : 0.0, (rr && lv1) ? qv.y * d.y : 0.0);
        const double2 v = dd((rr && lv0) ? sr.x * d.x : 0.0, (rr && lv1) ? sr.y * d.y : 0.0);
        U[m1] = u;
        V[m1] = v;
        if (q >= ib && q <= ie) {
          sv[1] += dot2(Z[m1], qv); // (z,q)
          sv[2] += dot2(qv, u);     // (q,u)
          sv[7] += dot2(qv, v);     // (q,v)
          sv[12] += dot2(sr, v);    // (s,v)
        }
      }
      // ---- F: row t-5 ----
      {
        const int q = t - 5;
        double2 d;
        const double2 au = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[5], bsl[4], U[m0], U[m2], U[m1], d);
        const double2 av = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[5], bsl[4], V[m0], V[m2], V[m1], d);
        const bool rr = interior(q);
        const double2 uu = dd((rr && lv0) ? au.x * d.x : 0.0, (rr && lv1) ? au.y * d.y : 0.0);
        const double2 vv = dd((rr && lv0) ? av.x * d.x : 0.0, (rr && lv1) ? av.y * d.y : 0.0);
        UU[m2] = uu;
        VV[m2] = vv;
        if (q >= ib && q <= ie) {
          const double2 u = U[m2], v = V[m2];
          sv[3] += dot2(u, au);    // (u,Au)
          sv[8] += dot2(u, av);    // (u,Av)
          sv[13] += dot2(v, av);   // (v,Av)
          sv[4] += dot2(au, uu);   // (Au,ũ)
          sv[9] += dot2(au, vv);   // (Au,ṽ)
          sv[14] += dot2(av, vv);  // (Av,ṽ)
        }
      }
      // ---- G: row t-6 ----
      {
        const int q = t - 6;
        if (q >= ib && q <= ie) {
          double2 d;
          const double2 auu = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[6], bsl[5], UU[m1], UU[m0], UU[m2], d);
          const double2 avv = apply_row<BAND>(k, rx, tvw, q, c0, jl, bsl[6], bsl[5], VV[m1], VV[m0], VV[m2], d);
          const double2 uu = UU[m0], vv = VV[m0];
          sv[5] += dot2(uu, auu);   // (ũ,Aũ)
          sv[10] += dot2(uu, avv);  // (ũ,Aṽ)
          sv[15] += dot2(vv, avv);  // (ṽ,Aṽ)
        }
      }
      bs = bs == kRing3 - 1 ? 0 : bs + 1;
    }
  }
  if constexpr (PUSH) {
    if (pushed) {  // delivered before this wave arrives anywhere
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
}

__device__ __forceinline__ Coef3 uni3(const Coef3& c) {
  Coef3 u;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    u.zc[i] = uni(c.zc[i]);
    u.a[i] = uni(c.a[i]);
    u.b[i] = uni(c.b[i]);
    u.cw[i] = uni(c.cw[i]);
  }
  return u;
}

// Walk this wave's positions of the static item list.
template <bool PUSH>
__device__ __forceinline__ void walk3(const KParams& k, const Coef3& cf, bool fix, int par, WaveTV3& tv, int wid,
                                      double (&acc)[NS]) {
  const int W = k.lwaves;
  for (int pos = int(blockIdx.x) * kWPB + wid; pos < k.nslots; pos += W) {
    const int2 e = cload_i2(k.ilist + pos);
    const int rows = e.y >> 20;
    if (rows == 0) continue;  // empty position of the static layout
    const int s = e.y & 0xFFFFF, ib = e.x & kRowMask;
    const int ie = min(ib + rows - 1, int(k.nx));
    if (e.x & kBandBit) march3<true, PUSH>(k, cf, fix, par, s, ib, ie, tv, acc);
    else march3<false, PUSH>(k, cf, fix, par, s, ib, ie, tv, acc);
  }
}

template <bool PUSH>
__global__ __launch_bounds__(TJ) __attribute__((amdgpu_waves_per_eu(1))) void kS3(KParams k, int par) {
  DevState* st = k.st;
  const int done = st->done;
  const int fix = st->fixpend;
  __shared__ double sm[4 * NS];
  __shared__ int sflag;
  __shared__ WaveTV3 tvs[kWPB];
  const int lane = int(threadIdx.x & 63);
  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  if ((done || k.mlimit < 0) && !fix) return;  // (mlimit < 0: a fix-up-only launch)
  double acc[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  Scal3 sc = {};
  if (fix) {
    sc.first = false;
    sc.m = 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      sc.c.zc[i] = st->sc3[i];
      sc.c.a[i] = st->sc3[3 + i];
      sc.c.b[i] = st->sc3[6 + i];
      sc.c.cw[i] = st->sc3[9 + i];
    }
  } else {
    sc = sweep3_scalars(k, st, par);
    if (sc.m == 0 && !sc.first) {  // iteration K+1 breaks down before its update
      if (arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
        sweep3_terminal(st, sc);
        __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
  }
  const Coef3 cf = uni3(sc.c);
  const int rpar = fix ? st->wpar : par;  // the fix-up re-reads the converging sweep's inputs
  {  // band ring: defined contents (the never-written column 128 of b0 and the
     // slots garbage pipeline-fill rows read stay finite)
    WaveTV3& tv = tvs[wid];
    for (int i = lane; i < kRing3 * 128; i += 64) (&tv.a0r[0][0])[i] = 0.0;
    for (int i = lane; i < kRing3 * 130; i += 64) (&tv.b0r[0][0])[i] = 0.0;
  }
  walk3<PUSH>(k, cf, fix != 0, rpar, tvs[wid], wid, acc);
  if (fix) {  // fix-up launch: w only; the last wave clears the request
    if (arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
      st->fixpend = 0;
      __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (lane < 3 || lane > 60)  // strip halo lanes: recomputed copies of the neighbouring strips' columns
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  block_reduce<NS, false>(acc, sm);
  if (publish_last<NS>(k.partial + NS * size_t(blockIdx.x), acc, &st->ticket[0], gridDim.x, &sflag)) {
    double t[NS];
    reduce_partials<NS>(k.partial, gridDim.x, t, sm);
    __shared__ double xv[NS + 1];
    __shared__ unsigned long long sseq;
    __shared__ int sok;
    if (k.xr.peers) {  // cross-rank sum of the 19 sums inside the sweep (P2P transport)
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
      sweep3_finalize(k, st, par, sc, t);
      __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

void launch_S3(const KParams& k, int par, hipStream_t s) {
  if (k.push) hipLaunchKernelGGL(kS3<true>, dim3(unsigned(k.nblocks)), dim3(TJ), 0, s, k, par);
  else hipLaunchKernelGGL(kS3<false>, dim3(unsigned(k.nblocks)), dim3(TJ), 0, s, k, par);
}

int resident_blocks_S3() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kS3<false>, TJ, 0) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  return n;
}

}  // namespace dev
}  // namespace pe
