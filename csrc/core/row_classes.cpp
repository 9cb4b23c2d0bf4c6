// Per-row coefficient class intervals for the on-the-fly fictitious-domain
// coefficients (used by the gfx950 kernels).
//
// For local row q the kernels need a(q,j), a(q+1,j), b(q,j), b(q,j+1).
// A vertical face {x = c, y ∈ [s_j, e_j]} lies fully inside D iff
// s_j ≥ -half(q) and e_j ≤ half(q) (half = ellipse chord half-width at c);
// then chord_len = e_j - s_j ≈ h2 and face_coef returns exactly 1.  It is
// fully outside iff e_j ≤ -half or s_j ≥ half; then chord_len = 0 and
// face_coef returns exactly 1/eps.  s_j, e_j are monotone in j, and the
// horizontal-face half-width halfB(j) is unimodal in j, so every such set is
// an interval found by binary search: O(nx log ny) setup instead of the
// reference's O(nx·ny) coefficient arrays (fic_reg_local,
// stage2-mpi/poisson_mpi_decomp.cpp:124-170).  The intervals are
// conservative — anything not provably interior/exterior is classified
// "boundary band" and evaluated exactly — so the classification never
// changes a coefficient value.
#include <algorithm>
#include <climits>
#include <vector>

#include "pe/device.hpp"

namespace pe {
namespace {

struct Iv {
  int64_t lo = 1, hi = 0;  // empty when lo > hi
  bool empty() const { return lo > hi; }
};

Iv meet(Iv a, Iv b) { return Iv{std::max(a.lo, b.lo), std::min(a.hi, b.hi)}; }
Iv shift(Iv a, int64_t d) { return a.empty() ? a : Iv{a.lo + d, a.hi + d}; }

// First index in [lo, hi] where pred turns true (pred monotone F..T); hi+1 if never.
template <class P>
int64_t first_true(int64_t lo, int64_t hi, P pred) {
  int64_t a = lo, b = hi + 1;
  while (a < b) {
    const int64_t m = a + (b - a) / 2;
    if (pred(m)) b = m;
    else a = m + 1;
  }
  return a;
}
// Last index in [lo, hi] where pred is true (pred monotone T..F); lo-1 if never.
template <class P>
int64_t last_true(int64_t lo, int64_t hi, P pred) {
  int64_t a = lo - 1, b = hi;
  while (a < b) {
    const int64_t m = b - (b - a) / 2;
    if (pred(m)) a = m;
    else b = m - 1;
  }
  return a;
}

}  // namespace

std::vector<int> row_classes(const double* colT, const double* rowT, int64_t rows_hi, int64_t cols_hi, int64_t lo) {
  const int64_t L = lo, H = cols_hi;  // row-table index range
  auto sA = [&](int64_t j) { return rowT[(j - lo) * 4 + 0]; };
  auto eA = [&](int64_t j) { return rowT[(j - lo) * 4 + 1]; };
  auto hB = [&](int64_t j) { return rowT[(j - lo) * 4 + 2]; };
  // Peak of the unimodal halfB(j).
  int64_t peak = L;
  for (int64_t j = L; j <= H; ++j)
    if (hB(j) > hB(peak)) peak = j;

  auto a_in = [&](int64_t q) {
    const double half = colT[(q - lo) * 4 + 0];
    if (half < 0) return Iv{};
    return Iv{first_true(L, H, [&](int64_t j) { return sA(j) >= -half; }),
              last_true(L, H, [&](int64_t j) { return eA(j) <= half; })};
  };
  auto a_notout = [&](int64_t q) {
    const double half = colT[(q - lo) * 4 + 0];
    if (half < 0) return Iv{};
    return Iv{first_true(L, H, [&](int64_t j) { return eA(j) > -half; }),
              last_true(L, H, [&](int64_t j) { return sA(j) < half; })};
  };
  // {j : halfB(j) ≥ T} (strict: >) for the unimodal halfB.
  auto b_level = [&](double T, bool strict) {
    auto ok = [&](int64_t j) { return strict ? hB(j) > T : hB(j) >= T; };
    if (!ok(peak)) return Iv{};
    return Iv{first_true(L, peak, ok), last_true(peak, H, ok)};
  };
  auto b_in = [&](int64_t q) {
    const double sB = colT[(q - lo) * 4 + 1], eB = colT[(q - lo) * 4 + 2];
    return b_level(std::max(-sB, eB), false);
  };
  auto b_notout = [&](int64_t q) {
    const double sB = colT[(q - lo) * 4 + 1], eB = colT[(q - lo) * 4 + 2];
    return b_level(std::max(-eB, sB), true);
  };

  std::vector<int> out(size_t(rows_hi - lo + 1) * 4, 0);
  for (int64_t q = lo; q <= rows_hi - 1; ++q) {
    const Iv bi = b_in(q);
    const Iv in = meet(meet(a_in(q), a_in(q + 1)), meet(bi, shift(bi, -1)));
    const Iv bn = b_notout(q);
    int64_t olo = INT_MAX / 2, ohi = INT_MIN / 2;
    for (const Iv& v : {a_notout(q), a_notout(q + 1), bn, shift(bn, -1)})
      if (!v.empty()) {
        olo = std::min(olo, v.lo);
        ohi = std::max(ohi, v.hi);
      }
    int* o = out.data() + (q - lo) * 4;
    o[0] = in.empty() ? 1 : int(in.lo);
    o[1] = in.empty() ? 0 : int(in.hi);
    o[2] = int(olo);
    o[3] = int(ohi);
  }
  return out;
}

std::vector<double> chord_tables(const Problem& P, const Block& blk, int64_t rows_hi, int64_t cols_hi, int64_t lo) {
  const double h1 = P.h1(), h2 = P.h2();
  std::vector<double> t((rows_hi - lo + 1) * 4 + (cols_hi - lo + 1) * 4, 0.0);
  double* col = t.data();
  double* row = t.data() + (rows_hi - lo + 1) * 4;
  for (int64_t li = lo; li <= rows_hi; ++li) {
    const int64_t gi = blk.i0 - 1 + li;
    const double x = P.A1 + gi * h1;  // x_i exactly as the reference forms it
    double* c = col + (li - lo) * 4;
    c[0] = chord_half_vertical(x - 0.5 * h1, P.cx, P.cy, P.sx);
    c[1] = x - 0.5 * h1;
    c[2] = x + 0.5 * h1;
    c[3] = x;
  }
  for (int64_t lj = lo; lj <= cols_hi; ++lj) {
    const int64_t gj = blk.j0 - 1 + lj;
    const double y = P.A2 + gj * h2;
    double* r = row + (lj - lo) * 4;
    r[0] = y - 0.5 * h2;
    r[1] = y + 0.5 * h2;
    r[2] = chord_half_horizontal(y - 0.5 * h2, P.cx, P.cy, P.sy);
    r[3] = y;
  }
  return t;
}

void host_coefficients(const Problem& P, const Block& blk, std::vector<double>& a, std::vector<double>& b,
                       std::vector<int>& cls) {
  // Host mirror of the kernels' cset(): class lookup, then exact face
  // coefficients only in the boundary band (tests compare with fic_reg).
  const std::vector<double> t = chord_tables(P, blk, blk.nx + 2, blk.ny + 2);
  const double* col = t.data();
  const double* row = t.data() + (blk.nx + 4) * 4;
  const std::vector<int> rc = row_classes(col, row, blk.nx + 2, blk.ny + 2);
  const double h1 = P.h1(), h2 = P.h2(), eps = P.eps(), inv_eps = 1.0 / eps;
  const int64_t R = blk.nx + 2, C = blk.ny + 2;
  a.assign(size_t(R * C), 0.0);
  b.assign(size_t(R * C), 0.0);
  cls.assign(size_t(R * C), 0);
  for (int64_t q = 0; q < R; ++q)
    for (int64_t lj = 0; lj < C; ++lj) {
      const int* c = rc.data() + (q + 1) * 4;
      const size_t at = size_t(q * C + lj);
      if (lj >= c[0] && lj <= c[1]) {
        a[at] = b[at] = 1.0;
        cls[at] = 0;
      } else if (lj < c[2] || lj > c[3]) {
        a[at] = b[at] = inv_eps;
        cls[at] = 1;
      } else {
        const double* rv = row + (lj + 1) * 4;
        const double* cv = col + (q + 1) * 4;
        a[at] = face_coef(chord_len(cv[0], rv[0], rv[1]), h2, eps);
        b[at] = face_coef(chord_len(rv[2], cv[1], cv[2]), h1, eps);
        cls[at] = 2;
      }
    }
}

}  // namespace pe
