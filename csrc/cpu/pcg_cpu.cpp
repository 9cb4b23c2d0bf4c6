// CPU backends: serial / OpenMP / multi-rank (thread or callback transport)
// Jacobi-PCG on one block of the 2D decomposition.
//
// This is the numerics oracle of the framework: with threads = 1 and a
// single rank it reproduces the reference's stage2 solver operation for
// operation (stage2-mpi/poisson_mpi_decomp.cpp:356-460: same assembly,
// same divide-by-h operator, same sequential sums, same stop test), so the
// published iteration counts (546 @400x600, 989 @800x1200, ...) come out
// exactly.  Differences from the reference are deliberate and structural:
// flat 64-bit-indexed fields instead of vector<vector> (quirks A11/A12),
// no per-iteration allocation, all four halo directions posted at once,
// and deterministic OpenMP reductions (fixed per-thread chunks combined in
// thread order) instead of `reduction(+:…)`.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <thread>

#include "pe/solver.hpp"

namespace pe {
namespace {

using clk = std::chrono::steady_clock;
inline double secs(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

struct Fields {
  std::vector<double> a, b, B, w, r, z, p, Ap;
  explicit Fields(int64_t n) : a(n, 0.0), b(n, 0.0), B(n, 0.0), w(n, 0.0), r(n, 0.0), z(n, 0.0),
                               p(n, 0.0), Ap(n, 0.0) {}
};

// Deterministic parallel sum over owned rows: thread t sums a fixed
// contiguous row range in row-major order; partials are combined in thread
// order.  With T = 1 this is exactly the reference's sequential loop.
template <class F>
double row_sum(const Block& blk, int T, F&& term) {
  if (T <= 1) {
    double s = 0.0;
    for (int64_t li = 1; li <= blk.nx; ++li)
      for (int64_t lj = 1; lj <= blk.ny; ++lj) s += term(blk.at(li, lj));
    return s;
  }
  std::vector<double> part(T, 0.0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const int nt = omp_get_num_threads();
    const int64_t lo = 1 + (blk.nx * t) / nt, hi = (blk.nx * (t + 1)) / nt;
    double s = 0.0;
    for (int64_t li = lo; li <= hi; ++li)
      for (int64_t lj = 1; lj <= blk.ny; ++lj) s += term(blk.at(li, lj));
    part[t] = s;
  }
  double s = 0.0;
  for (int t = 0; t < T; ++t) s += part[t];
  return s;
}

void assemble(const Problem& P, const Block& blk, Fields& f, int T) {
  const double h1 = P.h1(), h2 = P.h2(), eps = P.eps();
  // a, b on the block plus a 1-wide ring (reference :132-157).
#pragma omp parallel for schedule(static) num_threads(T) if (T > 1)
  for (int64_t li = 0; li <= blk.nx + 1; ++li) {
    const int64_t gi = blk.i0 - 1 + li;
    const double x = P.A1 + gi * h1;
    for (int64_t lj = 0; lj <= blk.ny + 1; ++lj) {
      const int64_t gj = blk.j0 - 1 + lj;
      const double y = P.A2 + gj * h2;
      const double la = seg_len_vertical(x - 0.5 * h1, y - 0.5 * h2, y + 0.5 * h2, P.cx, P.cy, P.sx);
      const double lb = seg_len_horizontal(y - 0.5 * h2, x - 0.5 * h1, x + 0.5 * h1, P.cx, P.cy, P.sy);
      f.a[blk.at(li, lj)] = face_coef(la, h2, eps);
      f.b[blk.at(li, lj)] = face_coef(lb, h1, eps);
    }
  }
  // RHS on owned nodes (reference :160-169).
#pragma omp parallel for schedule(static) num_threads(T) if (T > 1)
  for (int64_t li = 1; li <= blk.nx; ++li) {
    const double x = P.A1 + (blk.i0 - 1 + li) * h1;
    for (int64_t lj = 1; lj <= blk.ny; ++lj) {
      const double y = P.A2 + (blk.j0 - 1 + lj) * h2;
      f.B[blk.at(li, lj)] = in_ellipse(x, y, P.cx, P.cy) ? P.F : 0.0;
    }
  }
}

// Ap = A p on owned nodes (reference mat_A_local :194-213, same expression).
void apply_A(const Block& blk, const double* w, const double* a, const double* b, double* Aw,
             double h1, double h2, int T) {
  const int64_t pitch = blk.pitch;
#pragma omp parallel for schedule(static) num_threads(T) if (T > 1)
  for (int64_t li = 1; li <= blk.nx; ++li) {
    for (int64_t lj = 1; lj <= blk.ny; ++lj) {
      const int64_t c = blk.at(li, lj);
      const double Ax = -1.0 / h1 *
                        (a[c + pitch] * (w[c + pitch] - w[c]) / h1 - a[c] * (w[c] - w[c - pitch]) / h1);
      const double Ay = -1.0 / h2 * (b[c + 1] * (w[c + 1] - w[c]) / h2 - b[c] * (w[c] - w[c - 1]) / h2);
      Aw[c] = Ax + Ay;
    }
  }
}

// z = D^{-1} r (reference mat_D :219-232; D recomputed from a, b).
void apply_Dinv(const Block& blk, const double* r, const double* a, const double* b, double* z,
                double h1, double h2, int T) {
  const int64_t pitch = blk.pitch;
#pragma omp parallel for schedule(static) num_threads(T) if (T > 1)
  for (int64_t li = 1; li <= blk.nx; ++li) {
    for (int64_t lj = 1; lj <= blk.ny; ++lj) {
      const int64_t c = blk.at(li, lj);
      const double D = (a[c + pitch] + a[c]) / (h1 * h1) + (b[c + 1] + b[c]) / (h2 * h2);
      z[c] = (D != 0.0) ? r[c] / D : 0.0;
    }
  }
}

// Halo exchange of one field: contiguous rows for x-neighbours, packed
// columns for y-neighbours.  Global-edge halos are never written (they stay
// zero from allocation: Dirichlet), unlike the reference which re-zeroes
// them every iteration (quirk A9).
class HaloExchanger {
 public:
  explicit HaloExchanger(const Block& blk) : blk_(blk) {
    for (int d = 0; d < 4; ++d) {
      const int64_t n = (d < 2) ? blk.ny : blk.nx;
      send_[d].assign(n, 0.0);
      recv_[d].assign(n, 0.0);
    }
  }
  void run(double* f, HostComm& comm) {
    std::vector<Exchange> ex;
    for (int d = 0; d < 4; ++d) {
      if (!blk_.has(d)) continue;
      pack(f, d);
      ex.push_back(Exchange{d, blk_.nbr[d], send_[d].data(), recv_[d].data(),
                            int64_t(send_[d].size())});
    }
    comm.exchange(ex);
    for (int d = 0; d < 4; ++d)
      if (blk_.has(d)) unpack(f, d);
  }

 private:
  void pack(const double* f, int d) {
    auto& s = send_[d];
    if (d == LEFT || d == RIGHT) {
      const int64_t li = (d == LEFT) ? 1 : blk_.nx;
      for (int64_t lj = 1; lj <= blk_.ny; ++lj) s[lj - 1] = f[blk_.at(li, lj)];
    } else {
      const int64_t lj = (d == DOWN) ? 1 : blk_.ny;
      for (int64_t li = 1; li <= blk_.nx; ++li) s[li - 1] = f[blk_.at(li, lj)];
    }
  }
  void unpack(double* f, int d) {
    const auto& r = recv_[d];
    if (d == LEFT || d == RIGHT) {
      const int64_t li = (d == LEFT) ? 0 : blk_.nx + 1;
      for (int64_t lj = 1; lj <= blk_.ny; ++lj) f[blk_.at(li, lj)] = r[lj - 1];
    } else {
      const int64_t lj = (d == DOWN) ? 0 : blk_.ny + 1;
      for (int64_t li = 1; li <= blk_.nx; ++li) f[blk_.at(li, lj)] = r[li - 1];
    }
  }
  const Block& blk_;
  std::vector<double> send_[4], recv_[4];
};

}  // namespace

SolveResult cpu_pcg(const Problem& P, const Block& blk, HostComm& comm, const SolveOptions& opt,
                    std::vector<double>* w_out) {
  const auto t_start = clk::now();
  SolveResult res;
  res.backend = opt.threads > 1 ? "cpu-omp" : "cpu-serial";
  res.Px = blk.Px;
  res.Py = blk.Py;
  const int T = std::max(1, opt.threads);
  const double h1 = P.h1(), h2 = P.h2();
  const bool weighted = P.norm == Norm::Weighted;
  const int64_t max_iter = P.iter_cap();

  Fields f(blk.alloc);
  assemble(P, blk, f, T);
  HaloExchanger halo(blk);

  // Initial guess: w⁰ = 0 (reference :384) or a deterministic random field.
  if (opt.init == Init::Random) {
    for (int64_t li = 0; li <= blk.nx + 1; ++li)
      for (int64_t lj = 0; lj <= blk.ny + 1; ++lj)
        f.w[blk.at(li, lj)] = random_w0(blk.i0 - 1 + li, blk.j0 - 1 + lj, P.M, P.N, opt.seed, opt.init_amp);
    apply_A(blk, f.w.data(), f.a.data(), f.b.data(), f.Ap.data(), h1, h2, T);
    for (int64_t li = 1; li <= blk.nx; ++li)
      for (int64_t lj = 1; lj <= blk.ny; ++lj) {
        const int64_t c = blk.at(li, lj);
        f.r[c] = f.B[c] - f.Ap[c];
      }
    // w's halo ring is only used to form r⁰; clear it so updates stay owned.
  } else {
    f.r = f.B;
  }
  apply_Dinv(blk, f.r.data(), f.a.data(), f.b.data(), f.z.data(), h1, h2, T);
  f.p = f.z;
  // p's halo ring must come from the exchange (reference :392: p = z copies
  // whole matrices, whose halo is 0 before the first exchange).
  for (int64_t li = 0; li <= blk.nx + 1; ++li)
    for (int64_t lj = 0; lj <= blk.ny + 1; ++lj)
      if (li == 0 || lj == 0 || li == blk.nx + 1 || lj == blk.ny + 1) f.p[blk.at(li, lj)] = 0.0;

  const double* z = f.z.data();
  const double* r = f.r.data();
  double zr_old = row_sum(blk, T, [&](int64_t c) { return z[c] * r[c]; }) * h1 * h2;
  comm.allreduce_sum(&zr_old, 1);
  res.t.setup = secs(t_start, clk::now());

  const auto t_loop = clk::now();
  int64_t iter = 0;
  for (int64_t k = 1; k <= max_iter; ++k) {
    iter = k;
    auto t0 = clk::now();
    halo.run(f.p.data(), comm);
    auto t1 = clk::now();
    res.t.halo += secs(t0, t1);

    apply_A(blk, f.p.data(), f.a.data(), f.b.data(), f.Ap.data(), h1, h2, T);
    auto t2 = clk::now();
    res.t.gpu += secs(t1, t2);
    const double* Ap = f.Ap.data();
    const double* p = f.p.data();
    double den = row_sum(blk, T, [&](int64_t c) { return Ap[c] * p[c]; }) * h1 * h2;
    auto t3 = clk::now();
    res.t.dot += secs(t2, t3);
    comm.allreduce_sum(&den, 1);
    auto t4 = clk::now();
    res.t.reduce += secs(t3, t4);
    if (!std::isfinite(den) || !std::isfinite(zr_old)) {  // failure detection: NaN/Inf in the reduced scalars
      res.nonfinite = true;
      break;
    }
    if (std::fabs(den) < 1e-15) {
      res.breakdown = true;
      break;
    }
    const double alpha = zr_old / den;

    // Fused w, r update + local ‖Δw‖² (reference :418-427).
    double* w = f.w.data();
    double* rr = f.r.data();
    auto upd = [&](int64_t li_lo, int64_t li_hi) {
      double s = 0.0;
      for (int64_t li = li_lo; li <= li_hi; ++li)
        for (int64_t lj = 1; lj <= blk.ny; ++lj) {
          const int64_t c = blk.at(li, lj);
          const double w_old = w[c];
          w[c] = w_old + alpha * p[c];
          rr[c] -= alpha * Ap[c];
          const double d = w[c] - w_old;
          s += d * d;
        }
      return s;
    };
    double diff = 0.0;
    if (T <= 1) {
      diff = upd(1, blk.nx);
    } else {
      std::vector<double> part(T, 0.0);
#pragma omp parallel num_threads(T)
      {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        part[t] = upd(1 + (blk.nx * t) / nt, (blk.nx * (t + 1)) / nt);
      }
      for (int t = 0; t < T; ++t) diff += part[t];
    }
    auto t5 = clk::now();
    res.t.gpu += secs(t4, t5);

    apply_Dinv(blk, f.r.data(), f.a.data(), f.b.data(), f.z.data(), h1, h2, T);
    auto t6 = clk::now();
    res.t.prec += secs(t5, t6);
    double zr_new = row_sum(blk, T, [&](int64_t c) { return z[c] * r[c]; }) * h1 * h2;
    auto t7 = clk::now();
    res.t.dot += secs(t6, t7);
    comm.allreduce_sum(&zr_new, 1);
    comm.allreduce_sum(&diff, 1);
    auto t8 = clk::now();
    res.t.reduce += secs(t7, t8);
    const double gdiff = weighted ? std::sqrt(diff * h1 * h2) : std::sqrt(diff);
    res.last_diff = gdiff;
    if (opt.keep_history) res.history.push_back(gdiff);
    if (opt.log_every > 0 && comm.rank() == 0 && (k % opt.log_every) == 0)
      std::fprintf(stderr, "[pe] iter %lld  |dw| = %.6e  (z,r) = %.6e\n", (long long)k, gdiff, zr_new);
    if (gdiff < P.tol) {
      res.converged = true;
      zr_old = zr_new;
      break;
    }
    const double beta = zr_new / zr_old;
    zr_old = zr_new;
#pragma omp parallel for schedule(static) num_threads(T) if (T > 1)
    for (int64_t li = 1; li <= blk.nx; ++li)
      for (int64_t lj = 1; lj <= blk.ny; ++lj) {
        const int64_t c = blk.at(li, lj);
        f.p[c] = z[c] + beta * f.p[c];
      }
    res.t.gpu += secs(t8, clk::now());
  }
  res.iters = iter;
  res.zr = zr_old;
  res.t.iterate = secs(t_loop, clk::now());

  if (opt.compute_error) {
    double acc[1] = {0.0}, mx[2] = {0.0, 0.0};
    for (int64_t li = 1; li <= blk.nx; ++li) {
      const double x = P.A1 + (blk.i0 - 1 + li) * h1;
      for (int64_t lj = 1; lj <= blk.ny; ++lj) {
        const double y = P.A2 + (blk.j0 - 1 + lj) * h2;
        const double wv = f.w[blk.at(li, lj)];
        if (in_ellipse(x, y, P.cx, P.cy)) {
          const double u = P.u_scale() * (1.0 - P.cx * x * x - P.cy * y * y);
          const double e = wv - u;
          acc[0] += e * e;
          mx[0] = std::max(mx[0], std::fabs(e));
        } else {
          mx[1] = std::max(mx[1], std::fabs(wv));
        }
      }
    }
    comm.allreduce_sum(acc, 1);
    comm.allreduce_max(mx, 2);
    res.l2_err = std::sqrt(acc[0] * h1 * h2);
    res.max_err = mx[0];
    res.max_outside = mx[1];
  }
  if (w_out) {
    w_out->resize(size_t(blk.nx * blk.ny));
    for (int64_t li = 1; li <= blk.nx; ++li)
      for (int64_t lj = 1; lj <= blk.ny; ++lj)
        (*w_out)[size_t((li - 1) * blk.ny + (lj - 1))] = f.w[blk.at(li, lj)];
  }
  res.t.solver = secs(t_start, clk::now());
  return res;
}

SolveResult cpu_pcg_threads(const Problem& P, int ranks, DecompMode mode, const SolveOptions& opt,
                            std::vector<double>* w_out) {
  return cpu_pcg_threads(P, choose_process_grid(ranks, P.M, P.N, mode), opt, w_out);
}

SolveResult cpu_pcg_threads(const Problem& P, const ProcessGrid& pg, const SolveOptions& opt,
                            std::vector<double>* w_out) {
  const int ranks = pg.Px * pg.Py;
  auto group = make_thread_group(ranks);
  std::vector<SolveResult> results(ranks);
  std::vector<std::vector<double>> blocks(ranks);
  std::vector<Block> blks(ranks);
  std::vector<std::exception_ptr> errs(ranks);
  std::vector<std::thread> th;
  for (int r = 0; r < ranks; ++r) {
    blks[r] = decompose(P.M, P.N, pg, r);
    th.emplace_back([&, r] {
      try {
        auto comm = make_thread_comm(group, r);
        results[r] = cpu_pcg(P, blks[r], *comm, opt, w_out ? &blocks[r] : nullptr);
      } catch (...) {
        errs[r] = std::current_exception();
      }
    });
  }
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
  if (w_out) {
    const int64_t ny = P.N - 1;
    w_out->assign(size_t((P.M - 1) * ny), 0.0);
    for (int r = 0; r < ranks; ++r) {
      const Block& b = blks[r];
      for (int64_t li = 0; li < b.nx; ++li)
        for (int64_t lj = 0; lj < b.ny; ++lj)
          (*w_out)[size_t((b.i0 - 1 + li) * ny + (b.j0 - 1 + lj))] = blocks[r][size_t(li * b.ny + lj)];
    }
  }
  SolveResult out = results[0];
  // Timers: max over ranks (reference MPI_Reduce(MAX), poisson_mpi_cuda2.cu:962-966).
  for (int r = 1; r < ranks; ++r) {
    const Timers& t = results[r].t;
    out.t.gpu = std::max(out.t.gpu, t.gpu);
    out.t.halo = std::max(out.t.halo, t.halo);
    out.t.reduce = std::max(out.t.reduce, t.reduce);
    out.t.prec = std::max(out.t.prec, t.prec);
    out.t.dot = std::max(out.t.dot, t.dot);
    out.t.setup = std::max(out.t.setup, t.setup);
    out.t.solver = std::max(out.t.solver, t.solver);
    out.t.iterate = std::max(out.t.iterate, t.iterate);
  }
  out.backend = ranks > 1 ? (opt.threads > 1 ? "cpu-hybrid" : "cpu-ranks") : out.backend;
  return out;
}

}  // namespace pe
