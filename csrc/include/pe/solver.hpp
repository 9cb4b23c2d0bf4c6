// Solver options / results shared by every backend.
//
// Reference solvers: stage0 `solve` (Withoutopenmp1.cpp:106-172), stage1
// OpenMP `solve` (Withopenmp1.cpp:133-199), stage2/3 `solve_mpi`
// (poisson_mpi_decomp.cpp:356-460, main_hybrid.cpp:364-470) and the stage4
// GPU driver `gradient_solver_mpi` (poisson_mpi_cuda2.cu:687-982).  All of
// them are Jacobi-preconditioned CG with the stop rule ‖w^{k+1}-w^k‖_E < δ.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "pe/comm.hpp"
#include "pe/decomp.hpp"
#include "pe/problem.hpp"

namespace pe {

// Stage timers (seconds, this rank).  Categories follow the reference's
// stage-4 printout (poisson_mpi_cuda2.cu:955-979, timers :695-700) with
// honest semantics:
//   gpu     — device compute kernels (device solver: the sweep / stencil
//             kernels plus the reduction kernel; CPU solvers: the loops)
//   dot     — the dot-product reduction (device: the item-sum reduction
//             kernel, a subset of gpu — 0 and `dot_fused` when the fan-in
//             runs inside the sweep kernel itself)
//   copy    — host<->device copies (set-up tables, the per-chunk state read,
//             checkpoints; everything else is device-resident)
//   halo    — halo exchange (RCCL send/recv + unpack); 0 on one rank
//   reduce  — cross-rank allreduce launches (0 on one rank, or when the
//             sweep sums its scalars over ranks itself)
//   prec    — preconditioner (CPU solvers; fused into the device sweep)
//   setup   — construction (allocation, tables, item lists, placement
//             search) + initial state, before the first iteration
//   construct — the construction part of setup (device solver)
//   solver  — wall time of the whole solve: setup + iterations + error
//             (the reference's time_solver spans assembly, malloc, H2D, the
//             loop and free, poisson_mpi_cuda2.cu:1010-1016)
//   iterate — wall time of the iteration loop only
//   wait    — device solver, in-sweep cross-rank sum (P2P transport): the
//             time the sweeps' final blocks waited for the peers' flags
//             (s_memrealtime around the spin; it includes the halo push's
//             delivery, which those flags signal, and any rank imbalance —
//             what the reference's MPI_Allreduce time holds)
// Device solver: the per-phase device times come from hipEvent pairs around
// the phases of sampled iterations (no host sync in the loop; every
// PE_TIMER_SAMPLE-th chunk, default 8, its first two iterations; every
// iteration with SolveOptions::timing), scaled to the iterations run;
// `sampled` is the number of iterations measured.
struct Timers {
  double gpu = 0, copy = 0, halo = 0, reduce = 0, prec = 0, dot = 0, setup = 0, solver = 0;
  double iterate = 0;  // wall time of the iteration loop only
  double check = 0;    // the end-of-solve true-residual check (not in iterate / solver)
  double construct = 0, sampled = 0;
  double wait = 0;  // in-sweep cross-rank wait (see above)
  bool dot_fused = false;
};

struct SolveOptions {
  Init init = Init::Zero;
  uint64_t seed = 1234;
  double init_amp = 0.05;
  int threads = 1;           // CPU backends: OpenMP threads per rank
  int log_every = 0;         // >0: print ‖Δw‖ every K iterations (rank 0)
  bool keep_history = false; // record ‖Δw‖ of every iteration
  bool compute_error = true; // L2 / max error against the analytic solution
  bool verbose = false;
  // Device backend knobs.
  int chunk = 0;             // iterations enqueued per host check (0 = auto)
  // Capture a chunk of iterations into a hipGraph.  Off for solves: eager
  // launches keep up with the GPU (≥ 12 µs of kernel per iteration) and a
  // graph's instantiation pays the runtime's lazy copy-path set-up inside
  // T_solver (1600×2400: 0.126 vs 0.134-0.150 s, same µs / iteration,
  // profiles/r2_graph_ab.txt).  bench.py replays instantiated graphs.
  bool use_graph = false;
  bool timing = false;       // time every iteration's phases (default: a sample of them)
  bool check_tol = true;     // false: never stop on ‖Δw‖ (fixed-iteration benchmarking)
  int variant = 0;           // device arithmetic: 0 fast (1/h², 1/D), 1 reference expression trees
  // Device algorithm: 0 auto (single-sweep when the variant / decomposition
  // allow it), 1 classic two-kernel iteration (reference recurrence, 2
  // reductions), 2 single-sweep (fused.hip: 1 kernel, 1 reduction).
  int algo = 0;
  // Checkpoint / resume (device solver): every `checkpoint_every` iterations
  // (at the next chunk boundary) each rank writes `<checkpoint_path>.r<rank>`
  // (raw device state: fields, halo buffers, scalar block); `resume_path`
  // continues a solve from such files bitwise-identically.
  int64_t checkpoint_every = 0;
  std::string checkpoint_path;
  std::string resume_path;
};

struct SolveResult {
  int64_t iters = 0;
  bool converged = false;
  bool breakdown = false;
  bool nonfinite = false;  // a reduced scalar became NaN/Inf (device status 4)
  double last_diff = 0;  // ‖w^{k+1}-w^k‖ at the last iteration
  double zr = 0;         // final (z, r)
  Timers t;
  double l2_err = -1, max_err = -1, max_outside = -1;
  std::vector<double> history;
  int Px = 1, Py = 1;
  std::string backend;
  std::string algo;      // device: "fused" (single-sweep) or "classic"
  bool resident_fallback = false;  // device: a resident launch aborted, the solve finished on the streaming sweep
  // End-of-solve true-residual check (device single-sweep-layout paths; -1:
  // not computed): E-norms ‖B − A w‖ of the returned w, ‖B‖ and (three-step)
  // the recurrence's ‖r‖ of the same iterate and the relative gap
  // ‖B − A w − r‖ / ‖r‖; how many times the gap restarted the three-step
  // recurrence from w (residual replacement).
  double res_true = -1, res_rec = -1, res_gap = -1, b_norm = -1;
  int restarts = 0;
};

// ---- CPU backends (reference stage0..3 equivalents) -----------------------
// Reference-faithful PCG on one block of the decomposition; `comm` supplies
// halo exchange + reductions (SelfHostComm for serial/OpenMP runs).  When
// `w_out` is non-null the owned block of w is copied out row-major (nx × ny).
SolveResult cpu_pcg(const Problem& prob, const Block& blk, HostComm& comm,
                    const SolveOptions& opt, std::vector<double>* w_out = nullptr);

// Run P thread-ranks (ThreadHostComm) × `opt.threads` OpenMP threads each and
// return rank 0's result; `w_out` receives the gathered global interior
// ((M-1) × (N-1), row-major in i) when non-null.
SolveResult cpu_pcg_threads(const Problem& prob, int ranks, DecompMode mode,
                            const SolveOptions& opt, std::vector<double>* w_out = nullptr);
SolveResult cpu_pcg_threads(const Problem& prob, const ProcessGrid& pg, const SolveOptions& opt,
                            std::vector<double>* w_out = nullptr);

// Legacy-format report lines (reference stdout formats, §2.9 of SURVEY).
std::string format_result_legacy(const Problem& prob, const SolveResult& r, int nranks,
                                 const std::string& stage);

}  // namespace pe
