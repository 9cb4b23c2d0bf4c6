#include "pe/decomp.hpp"

#include <cmath>
#include <limits>
#include <sstream>
#include <stdexcept>

namespace pe {

ProcessGrid choose_process_grid_reference(int P) {
  // floor(sqrt(P)), decremented until it divides P (reference :60-64).
  ProcessGrid g;
  int Px = static_cast<int>(std::sqrt(static_cast<double>(P)));
  if (Px < 1) Px = 1;
  while (Px > 1 && P % Px != 0) --Px;
  g.Px = Px;
  g.Py = P / Px;
  return g;
}

double halo_cost(int M, int N, int Px, int Py) {
  // Per-rank worst-case bytes on the wire + a penalty for the strided
  // direction (needs pack/unpack passes).  Blocks are ceil-sized.
  const double nx = std::ceil(double(M - 1) / Px);
  const double ny = std::ceil(double(N - 1) / Py);
  const double xmsgs = Px > 1 ? (Px > 2 ? 2.0 : 1.0) : 0.0;
  const double ymsgs = Py > 1 ? (Py > 2 ? 2.0 : 1.0) : 0.0;
  return xmsgs * ny * 1.0 + ymsgs * nx * 1.5;
}

ProcessGrid choose_process_grid(int P, int M, int N, DecompMode mode) {
  if (P < 1) throw std::invalid_argument("process count must be >= 1");
  if (mode == DecompMode::Reference) return choose_process_grid_reference(P);
  if (mode == DecompMode::Rows) return ProcessGrid{P, 1};
  if (mode == DecompMode::Cols) return ProcessGrid{1, P};
  ProcessGrid best{P, 1};
  double best_cost = std::numeric_limits<double>::infinity();
  for (int Px = 1; Px <= P; ++Px) {
    if (P % Px) continue;
    const int Py = P / Px;
    if (Px > M - 1 || Py > N - 1) continue;
    const double c = halo_cost(M, N, Px, Py);
    if (c < best_cost - 1e-9) {
      best_cost = c;
      best = ProcessGrid{Px, Py};
    }
  }
  return best;
}

ProcessGrid process_grid_from_spec(const std::string& spec, int P, int M, int N) {
  if (spec == "reference") return choose_process_grid(P, M, N, DecompMode::Reference);
  if (spec == "aspect") return choose_process_grid(P, M, N, DecompMode::Aspect);
  if (spec == "rows") return choose_process_grid(P, M, N, DecompMode::Rows);
  if (spec == "cols") return choose_process_grid(P, M, N, DecompMode::Cols);
  // "device": the GPU solver's preference — P×1 row slabs while every rank
  // keeps >= 32 rows, else the aspect rule.  Both run the three-step sweep
  // (three iterations per pass); a slab's 6-row halo is one contiguous
  // message per side (no strided strips), a 2-D block adds the packed y
  // strips.  How it travels — the comm's RCCL exchange, the peer-put kernel
  // or (slabs) the sweep's own push, overlapped with the interior items or not
  // — the solver's construction decides by timing them on the job's transport
  // (DeviceSolver::choose_halo_path); the single sweep remains only for blocks
  // under 12 rows / columns.
  // Per rank block, zero-latency transport, measured with the two-step sweep
  // (profiles/r3_block_probe.txt): 4096² on 8 ranks 28.3 µs/iter as 8×1 vs
  // 39.8 as 4×2, on 4 ranks 41.2 vs 59.7 (4×1 / 2×2); 2048² on 8: 23.4 vs
  // 31.9; 16384² on 8: 168 vs 279.
  if (spec == "device") {
    if ((int64_t(M) - 1) / P >= 32) return choose_process_grid(P, M, N, DecompMode::Rows);
    return choose_process_grid(P, M, N, DecompMode::Aspect);
  }
  const auto x = spec.find('x');
  if (x == std::string::npos || x == 0 || x + 1 >= spec.size())
    throw std::invalid_argument("decomposition must be reference|aspect|rows|cols|device|<Px>x<Py>, got '" + spec + "'");
  ProcessGrid g{std::stoi(spec.substr(0, x)), std::stoi(spec.substr(x + 1))};
  if (g.Px < 1 || g.Py < 1 || g.Px * g.Py != P)
    throw std::invalid_argument("process grid " + spec + " does not match " + std::to_string(P) + " ranks");
  return g;
}

static void split_1d(int64_t total, int parts, int idx, int64_t& start, int64_t& count) {
  // Remainder to the lowest coordinates; sizes differ by at most 1 (reference :84-110).
  const int64_t base = total / parts, rem = total % parts;
  start = 1 + idx * base + std::min<int64_t>(idx, rem);
  count = base + (idx < rem ? 1 : 0);
}

Block decompose(int M, int N, const ProcessGrid& pg, int rank, int align) {
  if (pg.Px < 1 || pg.Py < 1) throw std::invalid_argument("bad process grid");
  if (rank < 0 || rank >= pg.Px * pg.Py) throw std::invalid_argument("rank out of range");
  if (M < 2 || N < 2) throw std::invalid_argument("grid must have M, N >= 2");
  if (align < 1) align = 1;
  Block b;
  b.rank = rank;
  b.size = pg.Px * pg.Py;
  b.Px = pg.Px;
  b.Py = pg.Py;
  b.px = rank % pg.Px;  // x-fastest rank order (reference :80-81)
  b.py = rank / pg.Px;
  int64_t cnt;
  split_1d(M - 1, pg.Px, b.px, b.i0, cnt);
  b.nx = cnt;
  b.i1 = b.i0 + cnt - 1;
  split_1d(N - 1, pg.Py, b.py, b.j0, cnt);
  b.ny = cnt;
  b.j1 = b.j0 + cnt - 1;
  b.rows = b.nx + 2;
  // Pad the pitch so every row's first owned element (lj = 1) is aligned.
  b.pitch = ((b.ny + 2 + align - 1) / align) * align;
  b.base = align - 1;  // (li, 1) → base + li*pitch + 1 ≡ 0 (mod align)
  // Two padding rows past the halo: the marching kernels prefetch up to
  // row nx+3 without clamping the address.
  b.alloc = b.base + (b.rows + 2) * b.pitch + align;
  b.nbr[LEFT] = b.px > 0 ? rank - 1 : -1;
  b.nbr[RIGHT] = b.px < pg.Px - 1 ? rank + 1 : -1;
  b.nbr[DOWN] = b.py > 0 ? rank - pg.Px : -1;
  b.nbr[UP] = b.py < pg.Py - 1 ? rank + pg.Px : -1;
  return b;
}

std::string describe(const Block& b) {
  std::ostringstream os;
  os << "rank " << b.rank << "/" << b.size << " grid " << b.Px << "x" << b.Py << " (" << b.px
     << "," << b.py << ") i=[" << b.i0 << "," << b.i1 << "] j=[" << b.j0 << "," << b.j1
     << "] nx=" << b.nx << " ny=" << b.ny << " pitch=" << b.pitch;
  return os.str();
}

}  // namespace pe
