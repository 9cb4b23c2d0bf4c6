// pe_cpu — CPU backends (the reference's stage0..stage3 executables as one
// configurable program).
//   pe_cpu [--backend serial|omp|ranks] [--ranks P] [--threads T]
//          [--threads-sweep 1,4,16] [--norm weighted|unweighted]
//          [--decomp reference|aspect] [--init zero|random] [--seed S]
//          [--tol 1e-6] [--max-iter K] [--stage stage0|stage1|stage2|stage3]
//          [--json] [M N]
// Replaces: stage0/Withoutopenmp*.cpp main (:176-196), stage1 thread sweep
// (Withopenmp2.cpp:204-229), stage2/3 mpirun runs (poisson_mpi_decomp.cpp:463-502,
// main_hybrid.cpp:473-512) — ranks are threads here (no MPI needed).
#include <cstdio>
#include <iostream>
#include <sstream>

#include "args.hpp"
#include "pe/solver.hpp"

using namespace pe;

static std::vector<int> parse_list(const std::string& s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, ','))
    if (!t.empty()) v.push_back(std::atoi(t.c_str()));
  return v;
}

int main(int argc, char** argv) {
  Args args(argc, argv);
  if (args.flag("help")) {
    std::puts("usage: pe_cpu [--backend serial|omp|ranks] [--ranks P] [--threads T] [--threads-sweep L]\n"
              "              [--norm weighted|unweighted] [--decomp reference|aspect] [--init zero|random]\n"
              "              [--seed S] [--tol D] [--max-iter K] [--stage stage0..3] [--grids 10,20,40] [--json] [M N]");
    return 0;
  }
  Problem P;
  const auto& pos = args.positional();
  if (pos.size() >= 2) {
    P.M = std::atoi(pos[0].c_str());
    P.N = std::atoi(pos[1].c_str());
  }
  P.tol = args.getd("tol", 1e-6);
  P.max_iter = args.geti("max-iter", -1);
  const std::string backend = args.get("backend", "serial");
  std::string stage = args.get("stage", "");
  // stage0 (Withoutopenmp1.cpp:106-196) stops on the unweighted ‖Δw‖ and, run
  // without M N, loops over the grids {10, 20, 40}² (:177)
  P.norm = args.get("norm", stage == "stage0" ? "unweighted" : "weighted") == "unweighted" ? Norm::Unweighted
                                                                                          : Norm::Weighted;
  std::vector<int> grids = parse_list(args.get("grids", (stage == "stage0" && pos.size() < 2) ? "10,20,40" : ""));
  int ranks = int(args.geti("ranks", 1));
  int threads = int(args.geti("threads", backend == "omp" ? 4 : 1));
  const std::string decomp = args.get("decomp", "reference");
  SolveOptions opt;
  opt.init = args.get("init", "zero") == "random" ? Init::Random : Init::Zero;
  opt.seed = uint64_t(args.geti("seed", 1234));
  opt.log_every = int(args.geti("log-every", 0));
  if (stage.empty()) stage = (backend != "serial" && backend != "omp" && threads > 1) ? "stage3" : "stage2";

  std::vector<int> sweep = parse_list(args.get("threads-sweep", ""));
  if (sweep.empty()) sweep.push_back(threads);
  if (backend != "ranks") ranks = 1;

  if (ranks > 1 || backend == "ranks")
    std::cout << (threads > 1 ? "MPI/OpenMP run with " : "Pure MPI 2D run with ") << ranks
              << (threads > 1 ? " MPI processes; " : " processes; ") << "M=" << P.M << ", N=" << P.N << std::endl;
  std::vector<std::pair<int, int>> sizes;
  for (int g : grids) sizes.emplace_back(g, g);
  if (sizes.empty()) sizes.emplace_back(P.M, P.N);
  for (const auto& mn : sizes)
  for (int t : sweep) {
    P.M = mn.first;
    P.N = mn.second;
    opt.threads = t;
    SolveResult r = cpu_pcg_threads(P, process_grid_from_spec(decomp, ranks, P.M, P.N), opt);
    if (args.flag("json")) {
      std::printf("{\"M\": %d, \"N\": %d, \"backend\": \"%s\", \"ranks\": %d, \"threads\": %d, \"Px\": %d, \"Py\": %d, "
                  "\"iters\": %lld, \"converged\": %s, \"t_solver\": %.6f, \"t_iterate\": %.6f, \"t_halo\": %.6f, "
                  "\"t_reduce\": %.6f, \"t_prec\": %.6f, \"t_dot\": %.6f, \"l2_err\": %.6e, \"max_err\": %.6e, "
                  "\"max_outside\": %.6e}\n",
                  P.M, P.N, r.backend.c_str(), ranks, t, r.Px, r.Py, (long long)r.iters,
                  r.converged ? "true" : "false", r.t.solver, r.t.iterate, r.t.halo, r.t.reduce, r.t.prec,
                  r.t.dot, r.l2_err, r.max_err, r.max_outside);
    } else {
      if (sweep.size() > 1) std::printf("Threads = %2d | Time = %.3f s | Iter=%lld\n", t, r.t.solver, (long long)r.iters);
      else std::cout << format_result_legacy(P, r, ranks, stage);
      std::printf("   L2 error in D ~ %.6e   max error in D ~ %.6e   max |w| outside D ~ %.3e\n", r.l2_err,
                  r.max_err, r.max_outside);
    }
  }
  return 0;
}
