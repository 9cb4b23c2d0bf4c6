// LDS-resident single-sweep Jacobi-PCG for small single-rank blocks: MANY
// iterations in ONE launch, the iterate never leaves the chip.
//
// Same Krylov recurrence as fused.hip (one 7-sum reduction per iteration;
// reference iteration: poisson_mpi_cuda2.cu:846-942), different machine
// mapping.  On blocks of ≲2 M nodes (the published 400×600 / 800×1200 grids,
// BASELINE.md §1) a streaming sweep is latency-bound: every wave gets about
// one item, so the kernel boundary, the prologue round trips and the item
// tail dominate (profiles/r2_tune.txt: 26 µs per iteration at 800×1200 where
// 40 B/node would stream in 8).  Here each workgroup owns one tile — a
// 124-column strip × R ≤ 64 rows — for the whole launch:
//
//   LDS   r and p of the tile plus a 2-deep ring (R+4 rows × 128 columns),
//         per-node coefficient codes (interior / exterior / band slot) and the
//         tile's boundary-band coefficients, evaluated once per launch;
//   VGPRs w of the wave's owned rows.
//
// Iteration k (every workgroup computes the same α_k, β_k from the previous
// iteration's 7 global sums):
//   A  p_k = D⁻¹ r + β p            on the whole region (ring included: the
//                                    ring of p needs no exchange, ever)
//   B  s = A p_k, r_k = r − α s,    on the tile + ring 1 (recomputed: equal
//      z_k = D⁻¹ r_k, 6 sums         bits to the owner's); r_k of the
//                                    neighbours' ring 2 is published here
//   C  q = A z_k, (z,q), w += α p_k  on the tile
//   →  7 partial sums published, ONE grid barrier, then every workgroup reads
//      the ring 2 of r from its 8 neighbours and ALL partial sums, and adds
//      them in a fixed order (the same bits everywhere: deterministic).
// Hand-off protocol (the image's CDNA4 guide /opt/skills/guides/MI355X_MICROARCH.md,
// not part of this repo: "Valid forms" row 1): every
// published value is stored `sc1` (relaxed agent-scope atomic store), each
// storing wave drains `vmcnt(0)`, a workgroup barrier, ONE lane adds to a
// per-XCD-sharded counter; consumers poll with `sc1` loads, barrier, and read
// every handed-off value with `sc1` loads.  A barrier wait that exceeds
// rp.timeout_ticks aborts the launch with status 5 (no hang).
//
// The launch starts from and ends in fused.hip's layout and state (x[b]
// r/p planes, w, DevState::fs / gprev / iter), so it interleaves freely with
// the streaming sweep (S_0, checkpoints, copy_w all unchanged), and the
// result does not depend on how iterations are split into launches.
#include "kcommon.hpp"

#pragma clang fp contract(fast)

namespace pe {
namespace dev {

namespace {

constexpr int RT = kResThreads;
constexpr int RW = RT / 64;               // waves
constexpr int RWR = kResMaxRows / RW;     // owned rows per wave in phase C (w registers)
constexpr int EROWT = 0, EROWB = kFSW, ECOLL = 2 * kFSW, ECOLR = 2 * kFSW + kResMaxRows;
static_assert(ECOLR + kResMaxRows == kResEdge, "edge record layout");

typedef double d2 __attribute__((ext_vector_type(2)));  // (HIP's double2 has no address-space-3 operators)
__device__ __forceinline__ d2 dd(double a, double b) { return d2{a, b}; }
__device__ __forceinline__ int lo16(int v) { return int(short(v & 0xFFFF)); }
__device__ __forceinline__ int hi16(int v) { return v >> 16; }

// sc1 (L2-coherent, write-through) stores and loads of handed-off values
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// LDS pointers carry address space 3 explicitly: derived through a struct or
// a select, a generic pointer compiles to flat loads that wait on vmcnt too.
#define LDS __attribute__((address_space(3)))

struct Coef {
  double inv_eps, ih1sq, ih2sq;
  const LDS double* band;  // [4][cap]: a0, a1, b0, b1 of the tile's boundary-band nodes
  int cap;
  // (A u) at a node: plain nodes f·Δu (f = 1 inside, 1/eps outside), band
  // nodes the general 5-point form (fused.hip: lapf / stencil<false>)
  __device__ __forceinline__ double apply(int code, double um, double u0, double un, double ul, double ur) const {
    if (code >= 0) {
      const double a0 = band[code], a1 = band[cap + code], b0 = band[2 * cap + code], b1 = band[3 * cap + code];
      return (a0 * (u0 - um) - a1 * (un - u0)) * ih1sq + (b0 * (u0 - ul) - b1 * (ur - u0)) * ih2sq;
    }
    const double f = code == -1 ? 1.0 : inv_eps;
    return f * (((u0 - um) - (un - u0)) * ih1sq + ((u0 - ul) - (ur - u0)) * ih2sq);
  }
};

// (wave_sum63: kcommon.hpp)

__global__ __launch_bounds__(RT, 1) void kResident(KParams k, ResParams rp) {
  extern __shared__ double lds_raw[];
  DevState* st = k.st;
  const int tid = int(threadIdx.x), lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = int(blockIdx.x);
  const int tr = wg / rp.nstrips, s = wg - tr * rp.nstrips;
  const int I0 = rp.rowstart[tr], R = rp.rowstart[tr + 1] - I0;
  const int I0m = tr > 0 ? rp.rowstart[tr - 1] : 0;  // band tr-1's first row (ring-column imports)
  const int J0 = 1 + kFSW * s;
  const int nx = int(k.nx), ny = int(k.ny);
  const int wS = min(kFSW, ny - J0 + 1);  // owned columns of this strip
  const int RR = R + 4;                   // region rows (tile + 2-deep ring)
  const int rc4 = rp.rcap + 4;
  LDS d2* Rp = (LDS d2*)(lds_raw);
  LDS d2* Pp = Rp + rc4 * 64;
  LDS d2* Dp = Pp + rc4 * 64;  // 1/D of every region node (plain or band)
  LDS int* Cd = (LDS int*)(Dp + rc4 * 64);
  LDS double* band = (LDS double*)(Cd + rc4 * 64);
  LDS double* red = band + 4 * rp.nbcap;  // [RW][8] per-wave sums, [8] broadcast of the global sums
  LDS unsigned* misc = (LDS unsigned*)(red + RW * 8 + 8);  // band count, abort, overflow
  LDS double* Rd = (LDS double*)(Rp);
  const Coef cf{k.inv_eps, k.ih1sq, k.ih2sq, band, rp.nbcap};

  // ---- state of the previous iteration (fused.hip's DevState) ----
  const int done0 = st->done;
  const int wpend = st->wpend;
  const double alpha_st = st->alpha;
  double gprev = st->gprev;
  long long iter = st->iter;
  double S[7];
#pragma unroll
  for (int n = 0; n < 7; ++n) S[n] = st->fs[rp.par0 ^ 1][n];
  if (tid == 0) misc[0] = misc[1] = misc[2] = 0;
  // every thread's state reads have returned before this workgroup counts
  // itself in: workgroup 0 writes a terminal state of the launch's FIRST
  // iteration only once all workgroups are counted (none can then read a
  // half-written state or a premature `done`)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (done0) return;  // uniform: the solve has ended
  if (tid == 0) __hip_atomic_fetch_add(rp.ctr + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the terminal write of iteration 0 (workgroup 0, thread 0): wait for every
  // workgroup's entry (co-resident grid; the barrier timeout bounds it)
  auto entered_all = [&]() {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(rp.ctr + 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < unsigned(rp.nwg)) {
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > rp.timeout_ticks) break;
      __builtin_amdgcn_s_sleep(1);
    }
  };

  // ---- load the region, evaluate the coefficient codes ----
  const int c0 = J0 - 2 + 2 * lane;  // this lane's column pair (c0, c0+1) = region columns 2·lane, 2·lane+1
  const double* xin = k.x[rp.par0 ^ 1];
  for (int rho = wv; rho < RR; rho += RW) {
    const int t = I0 - 2 + rho;
    const double* row = xin + int64_t(t) * k.pitch + c0;
    Rp[rho * 64 + lane] = *reinterpret_cast<const d2*>(row);
    Pp[rho * 64 + lane] = *reinterpret_cast<const d2*>(row + k.poff);
    const int4 rv = *reinterpret_cast<const int4*>(k.rowcls + (t + 1) * 4);
    const RowCls rc{rv.x, rv.y, rv.z, rv.w};
    int code[2];
    double dv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int lj = c0 + h;
      if (lj >= rc.in_lo && lj <= rc.in_hi) {
        code[h] = -1;
        dv[h] = k.dinv_in;
      } else if (lj < rc.out_lo || lj > rc.out_hi) {
        code[h] = -2;
        dv[h] = k.dinv_out;
      } else {
        const unsigned slot = __hip_atomic_fetch_add(&misc[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (slot >= unsigned(rp.nbcap)) {
          misc[2] = 1;
          code[h] = -2;
          dv[h] = k.dinv_out;
        } else {
          const double* ctr = k.colT + (t + 1) * 4;
          const CT ct{ctr[0], ctr[4], ctr[1], ctr[2]};
          const double* tv = k.rowT + (lj + 1) * 4;
          const CS x = cset_rc(k, rc, ct, lj, TV{tv[0], tv[1], tv[2], tv[6]});
          band[slot] = x.a0;
          band[rp.nbcap + slot] = x.a1;
          band[2 * rp.nbcap + slot] = x.b0;
          band[3 * rp.nbcap + slot] = x.b1;
          code[h] = int(slot);
          dv[h] = x.d;
        }
      }
    }
    Cd[rho * 64 + lane] = (code[0] & 0xFFFF) | (code[1] << 16);
    Dp[rho * 64 + lane] = dd(dv[0], dv[1]);
  }
  // w of this wave's owned rows (phase C rows cb0 .. cb1-1), with a pending
  // α·p term of a deferring streaming sweep applied (= kWFlush)
  const int cb0 = 2 + (R * wv) / RW, cb1 = 2 + (R * (wv + 1)) / RW;
  const bool ow0 = 2 * lane >= 2 && 2 * lane < 2 + wS;
  const bool ow1 = 2 * lane + 1 >= 2 && 2 * lane + 1 < 2 + wS;
  d2 wr[RWR];
#pragma unroll
  for (int q = 0; q < RWR; ++q) {
    wr[q] = dd(0.0, 0.0);
    const int rho = cb0 + q;
    if (rho < cb1) {
      const int t = I0 - 2 + rho;
      d2 w = *reinterpret_cast<const d2*>(k.w + int64_t(t) * k.wpitch + c0);
      if (wpend) {
        const d2 p = *reinterpret_cast<const d2*>(xin + int64_t(t) * k.pitch + k.poff + c0);
        w = dd(w.x + alpha_st * p.x, w.y + alpha_st * p.y);
      }
      wr[q] = w;
    }
  }
  __syncthreads();
  if (misc[2]) {  // band table overflow: the host sizes it, so this is an internal error
    if (tid == 0) {
      st->status = 5;
      st->done = 1;
    }
    return;
  }

  const double hh = k.h1 * k.h2;
  double g = 0.0, alpha = 0.0, beta = 0.0, diff = 0.0;
  bool stopped = false;
  int it = 0;
  unsigned long long* stp = nullptr;
  auto stamp = [&](int j) {
    if (stp && tid == 0) stp[j] = rtc();
  };
  for (; it < rp.niter; ++it) {
    const int buf = it & 1;
    stp = (rp.stamps && it < kResStampIters) ? rp.stamps + (size_t(wg) * kResStampIters + it) * 8 : nullptr;
    stamp(0);
    const long long kiter = iter + 1;
    // ---- scalars (fused.hip sweep_scalars / sweep_term, iterations only) ----
    g = S[0] * hh;
    beta = iter == 0 ? 0.0 : g / gprev;
    const double den = S[1] * hh + 2.0 * beta * (S[2] * hh) + beta * beta * (S[3] * hh);
    alpha = g / den;
    const double pn2 = fmax(S[4] + 2.0 * beta * S[5] + beta * beta * S[6], 0.0);
    diff = k.weighted ? fabs(alpha) * sqrt(pn2 * hh) : fabs(alpha) * sqrt(pn2);
    const bool tiny = fabs(den) < 1e-15;  // breakdown before α (reference :413)
    const bool bad = !isfinite(den) || !isfinite(g) || (!tiny && !isfinite(diff));
    const bool brk = bad || tiny;
    const bool conv = k.check_tol && diff < k.tol;
    const bool last = !brk && (conv || kiter >= k.max_iter);
    if (brk) {  // reference :413 — stop before this iteration's update
      if (wg == 0 && tid == 0) {
        if (it == 0) entered_all();
        st->status = bad ? 4 : 2;
        st->iter = kiter;
        st->done = 1;
        st->wpend = 0;
      }
      stopped = true;
      break;
    }

    // ---- A: p_k on the region (two rows per step, loads first) ----
    for (int rho = wv; rho < RR; rho += 2 * RW) {
      const int r2 = min(rho + RW, RR - 1);  // second row (a duplicate of the first past the end)
      const d2 ra = Rp[rho * 64 + lane], pa = Pp[rho * 64 + lane], da = Dp[rho * 64 + lane];
      const d2 rb = Rp[r2 * 64 + lane], pb = Pp[r2 * 64 + lane], db = Dp[r2 * 64 + lane];
      const d2 na = dd(ra.x * da.x + beta * pa.x, ra.y * da.y + beta * pa.y);
      const d2 nb = dd(rb.x * db.x + beta * pb.x, rb.y * db.y + beta * pb.y);
      Pp[rho * 64 + lane] = na;
      if (rho + RW < RR) Pp[r2 * 64 + lane] = nb;
    }
    __syncthreads();
    stamp(1);
    if (last) {  // converged / iteration cap: only w changes (w += α_k p_k)
#pragma unroll
      for (int q = 0; q < RWR; ++q) {
        const int rho = cb0 + q;
        if (rho < cb1) {
          const d2 p = Pp[rho * 64 + lane];
          wr[q] = dd(wr[q].x + alpha * p.x, wr[q].y + alpha * p.y);
        }
      }
      if (wg == 0 && tid == 0) {
        if (it == 0) entered_all();
        st->gprev = g;
        st->rz_cur = g;
        st->alpha = alpha;
        st->beta = beta;
        st->last_diff = diff;
        if (k.hist && kiter <= k.hist_n) k.hist[kiter - 1] = diff;
        st->iter = kiter;
        st->status = conv ? 1 : 3;
        st->done = 1;
        st->wpend = 0;
      }
      stopped = true;
      break;
    }

    // ---- B: s = A p_k, r_k, z_k on tile + ring 1; 6 sums; ring-2 edges ----
    // (software-pipelined march: the next row's operands are read before
    // this row's arithmetic)
    double sg = 0.0, sd = 0.0, se = 0.0, sps = 0.0, szz = 0.0, szp = 0.0, spp = 0.0;
    double* E = rp.edges + (size_t(buf) * size_t(rp.nwg) + size_t(wg)) * kResEdge;
    {
      const int nB = R + 2;
      const int b0 = 1 + (nB * wv) / RW, b1 = 1 + (nB * (wv + 1)) / RW;
      if (b0 < b1) {
        d2 pm = Pp[(b0 - 1) * 64 + lane], p0 = Pp[b0 * 64 + lane], pn = Pp[(b0 + 1) * 64 + lane];
        d2 r = Rp[b0 * 64 + lane], dv = Dp[b0 * 64 + lane];
        int cd = Cd[b0 * 64 + lane];
        for (int rho = b0; rho < b1; ++rho) {
          const int nr = min(rho + 1, b1 - 1);
          const d2 pnn = Pp[(nr + 1) * 64 + lane];
          const d2 rn = Rp[nr * 64 + lane], dvn = Dp[nr * 64 + lane];
          const int cdn = Cd[nr * 64 + lane];
          const int cA = lo16(cd), cB = hi16(cd);
          const double pl = dpp_shr1(p0.y), pr = dpp_shl1(p0.x);
          const double s0 = cf.apply(cA, pm.x, p0.x, pn.x, pl, p0.y);
          const double s1 = cf.apply(cB, pm.y, p0.y, pn.y, p0.x, pr);
          const int t = I0 - 2 + rho;
          const bool rl = t >= 1 && t <= nx;
          const bool lv0 = rl && lane >= 1 && c0 >= 1 && c0 <= ny;            // ring 2 columns excluded
          const bool lv1 = rl && lane <= 62 && c0 + 1 >= 1 && c0 + 1 <= ny;
          const double rk0 = lv0 ? r.x - alpha * s0 : r.x;
          const double rk1 = lv1 ? r.y - alpha * s1 : r.y;
          Rp[rho * 64 + lane] = dd(rk0, rk1);
          if (rho >= 2 && rho < R + 2) {  // owned row
            const double z0v = rk0 * dv.x, z1v = rk1 * dv.y;
            const double zo0 = ow0 ? z0v : 0.0, zo1 = ow1 ? z1v : 0.0;
            const double po0 = ow0 ? p0.x : 0.0, po1 = ow1 ? p0.y : 0.0;
            sg += rk0 * zo0 + rk1 * zo1;
            se += zo0 * s0 + zo1 * s1;
            sps += po0 * s0 + po1 * s1;
            szz += zo0 * zo0 + zo1 * zo1;
            szp += zo0 * po0 + zo1 * po1;
            spp += po0 * po0 + po1 * po1;
            // the neighbours' ring 2: tile rows 1 and R-2, tile columns 1 and 122
            if (rho == 3) {
              if (ow0) st_sc1(E + EROWT + 2 * lane - 2, rk0);
              if (ow1) st_sc1(E + EROWT + 2 * lane - 1, rk1);
            }
            if (rho == R) {
              if (ow0) st_sc1(E + EROWB + 2 * lane - 2, rk0);
              if (ow1) st_sc1(E + EROWB + 2 * lane - 1, rk1);
            }
            if (lane == 1 && ow1) st_sc1(E + ECOLL + rho - 2, rk1);
            if (lane == 62 && ow0) st_sc1(E + ECOLR + rho - 2, rk0);
          }
          pm = p0;
          p0 = pn;
          pn = pnn;
          r = rn;
          dv = dvn;
          cd = cdn;
        }
      }
    }
    __syncthreads();
    stamp(2);

    // ---- C: q = A z_k, (z, q), w += α p_k on the tile (pipelined march) ----
    {
      if (cb0 < cb1) {
        auto zr = [&](int rho) {
          const d2 r = Rp[rho * 64 + lane], d = Dp[rho * 64 + lane];
          return dd(r.x * d.x, r.y * d.y);
        };
        d2 zm = zr(cb0 - 1), z0 = zr(cb0);
        d2 rn = Rp[(cb0 + 1) * 64 + lane], dn = Dp[(cb0 + 1) * 64 + lane];
        int c0d = Cd[cb0 * 64 + lane];
        d2 pv = Pp[cb0 * 64 + lane];
#pragma unroll
        for (int q = 0; q < RWR; ++q) {
          const int rho = cb0 + q;
          if (rho >= cb1) break;
          const int nr = min(rho + 1, cb1 - 1);
          const d2 rnn = Rp[(nr + 1) * 64 + lane], dnn = Dp[(nr + 1) * 64 + lane];
          const int cdn = Cd[nr * 64 + lane];
          const d2 pvn = Pp[nr * 64 + lane];
          const d2 zn = dd(rn.x * dn.x, rn.y * dn.y);
          const double zl = dpp_shr1(z0.y), zrr = dpp_shl1(z0.x);
          const double q0 = cf.apply(lo16(c0d), zm.x, z0.x, zn.x, zl, z0.y);
          const double q1 = cf.apply(hi16(c0d), zm.y, z0.y, zn.y, z0.x, zrr);
          const double zo0 = ow0 ? z0.x : 0.0, zo1 = ow1 ? z0.y : 0.0;
          sd += zo0 * q0 + zo1 * q1;
          wr[q] = dd(wr[q].x + alpha * pv.x, wr[q].y + alpha * pv.y);
          zm = z0;
          z0 = zn;
          c0d = cdn;
          rn = rnn;
          dn = dnn;
          pv = pvn;
        }
      }
    }

    // ---- this tile's 7 sums (transposed: wave n < 7 sums quantity n) →
    //      published; grid barrier ----
    {
      double v[7] = {sg, sd, se, sps, szz, szp, spp};
#pragma unroll
      for (int n = 0; n < 7; ++n) v[n] = wave_sum63(v[n]);
      if (lane == 63)
#pragma unroll
        for (int n = 0; n < 7; ++n) red[wv * 8 + n] = v[n];
      __syncthreads();
      stamp(3);
      if (wv < 7 && lane == 0) {  // wave n publishes quantity n (waves in order)
        double a = red[wv];
#pragma unroll
        for (int w = 1; w < RW; ++w) a += red[w * 8 + wv];
        st_sc1(rp.partials + (size_t(buf) * size_t(rp.nwg) + size_t(wg)) * 8 + wv, a);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
      __syncthreads();
      stamp(4);
      if (wv == 0) {
        if (it == 0 && wg == rp.fault_wg && rp.fault_late) {  // (fault hook: arrive after the others time out)
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < rp.timeout_ticks + rp.timeout_ticks / 2)
            __builtin_amdgcn_s_sleep(8);
        }
        if (lane == 0 && !(it == 0 && wg == rp.fault_wg && !rp.fault_late))  // (fault hook: one workgroup never arrives)
          __hip_atomic_fetch_add(rp.ctr + (wg & 7) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int x = lane & 7;
        const unsigned want = unsigned(it + 1) * unsigned((rp.nwg - x + 7) / 8);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = true;
        for (;;) {
          const unsigned v =
              lane < 8 ? __hip_atomic_load(rp.ctr + x * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : want;
          if (__all(v >= want)) break;
          if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > rp.timeout_ticks) {
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (!ok && lane == 0) misc[1] = 1;
      }
      __syncthreads();
      stamp(5);
    }
    if (misc[1]) {  // a peer never arrived: abort the solve (status 5).  A late peer may
                    // still pass the barrier and write its tile back: the host restarts the
                    // solve from scratch on the sticky res_abort, never resumes this state
      if (tid == 0) {
        st->status = 5;
        st->done = 1;
        __hip_atomic_store(&st->res_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }

    // ---- every tile's partial sums (wave n < 7: quantity n over ≤ 256
    //      tiles — setup_resident refuses larger grids, kResMaxTiles), ring 2
    //      of r (wave 7) ----
    if (wv < 7) {
      const double* P = rp.partials + size_t(buf) * size_t(rp.nwg) * 8 + wv;
      double v[4];
      static_assert(kResMaxTiles == 4 * 64, "gather width");
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = j * 64 + lane;
        v[j] = t < rp.nwg ? ld_sc1(P + size_t(t) * 8) : 0.0;
      }
      double a = ((v[0] + v[1]) + v[2]) + v[3];
      a = wave_sum63(a);
      if (lane == 63) {
        if (k.fault_iter > 0 && kiter == k.fault_iter && wv == 1) a = __builtin_nan("");  // PE_FAULT_INJECT=nan@iter:K
        red[RW * 8 + wv] = a;
      }
    } else {
      const double* Eb = rp.edges + size_t(buf) * size_t(rp.nwg) * kResEdge;
      // ring rows I0-2 (band tr-1's row R'-2) and I0+R+1 (band tr+1's row 1)
      double rv[4];
      int ridx[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool top = u < 2;
        const int h = u & 1;
        const int t = top ? I0 - 2 : I0 + R + 1;
        const int trs = top ? tr - 1 : tr + 1;
        const int c = c0 + h;
        ridx[u] = -1;
        rv[u] = 0.0;
        if (trs >= 0 && trs < rp.ntr && t >= 1 && t <= nx && c >= 1 && c <= ny) {
          const int s2 = c < J0 ? s - 1 : (c >= J0 + kFSW ? s + 1 : s);
          rv[u] = ld_sc1(Eb + size_t(trs * rp.nstrips + s2) * kResEdge + (top ? EROWB : EROWT) + (c - 1 - kFSW * s2));
          ridx[u] = (top ? 0 : R + 3) * 128 + 2 * lane + h;
        }
      }
      // ring columns J0-2 (strip s-1's column 122) and J0+125 (strip s+1's column 1)
      double cv[4];
      int cidx[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool left = u < 2;
        const int rho = 1 + lane + 64 * (u & 1);
        const int c = left ? J0 - 2 : J0 + kFSW + 1;
        const int s2 = left ? s - 1 : s + 1;
        const int t = I0 - 2 + rho;
        cidx[u] = -1;
        cv[u] = 0.0;
        if (rho < R + 3 && s2 >= 0 && s2 < rp.nstrips && c >= 1 && c <= ny && t >= 1 && t <= nx) {
          const int trs = t < I0 ? tr - 1 : (t >= I0 + R ? tr + 1 : tr);
          const int idx = t - (t < I0 ? I0m : (t >= I0 + R ? I0 + R : I0));
          cv[u] = ld_sc1(Eb + size_t(trs * rp.nstrips + s2) * kResEdge + (left ? ECOLR : ECOLL) + idx);
          cidx[u] = rho * 128 + (left ? 0 : 127);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ridx[u] >= 0) Rd[ridx[u]] = rv[u];
        if (cidx[u] >= 0) Rd[cidx[u]] = cv[u];
      }
    }
    __syncthreads();
    stamp(6);
#pragma unroll
    for (int n = 0; n < 7; ++n) S[n] = red[RW * 8 + n];
    stamp(7);
    if (wg == 0 && tid == 0 && k.hist && kiter <= k.hist_n) k.hist[kiter - 1] = diff;
    gprev = g;
    iter = kiter;
  }

  // ---- write back: w always; r_k, p_k and the state after a full launch ----
#pragma unroll
  for (int q = 0; q < RWR; ++q) {
    const int rho = cb0 + q;
    if (rho < cb1) {
      double* wd = k.w + int64_t(I0 - 2 + rho) * k.wpitch + c0;
      if (ow0 && ow1) *reinterpret_cast<d2*>(wd) = wr[q];
      else if (ow0) wd[0] = wr[q].x;
      else if (ow1) wd[1] = wr[q].y;
    }
  }
  if (stopped) return;
  const int parl = (rp.par0 + rp.niter - 1) & 1;
  double* xo = k.x[parl];
  for (int rho = 2 + wv; rho < R + 2; rho += RW) {
    double* row = xo + int64_t(I0 - 2 + rho) * k.pitch + c0;
    const d2 r = Rp[rho * 64 + lane], p = Pp[rho * 64 + lane];
    if (ow0 && ow1) {
      *reinterpret_cast<d2*>(row) = r;
      *reinterpret_cast<d2*>(row + k.poff) = p;
    } else if (ow0) {
      row[0] = r.x;
      row[k.poff] = p.x;
    } else if (ow1) {
      row[1] = r.y;
      row[k.poff + 1] = p.y;
    }
  }
  if (wg == 0 && tid == 0) {
#pragma unroll
    for (int n = 0; n < 7; ++n) st->fs[parl][n] = S[n];
    st->gprev = g;
    st->rz_cur = g;
    st->alpha = alpha;
    st->beta = beta;
    st->last_diff = diff;
    st->iter = iter;
    st->started = 1;
    st->wpend = 0;
    st->wpar = parl;
  }
}

}  // namespace

size_t resident_lds_bytes(int rcap, int nbcap) {
  const size_t rc4 = size_t(rcap) + 4;
  return rc4 * 64 * 16 * 3 + rc4 * 64 * 4 + size_t(nbcap) * 4 * 8 + size_t(RW * 8 + 8) * 8 + 16;
}

int resident_max_blocks_per_cu(size_t lds_bytes) {
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kResident), hipFuncAttributeMaxDynamicSharedMemorySize,
                          int(lds_bytes)) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kResident, RT, lds_bytes) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

void launch_resident(const KParams& k, const ResParams& rp, hipStream_t s) {
  hipLaunchKernelGGL(kResident, dim3(unsigned(rp.nwg)), dim3(RT), rp.lds_bytes, s, k, rp);
}

}  // namespace dev
}  // namespace pe
