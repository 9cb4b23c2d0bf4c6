// pe_hip — the stage-4 executable (MPI + CUDA in the reference) rebuilt for
// MI355X: one process per GPU, RCCL over xGMI, device-resident PCG.
//
//   pe_hip [--tol 1e-6] [--max-iter K] [--decomp device|aspect|reference|rows|cols|PxxPy]
//          [--init zero|random] [--seed S] [--variant 0|1] [--algo auto|classic|fused|two-step|three-step] [--chunk K]
//          [--graph] [--timing] [--vranks P] [--json] [M N]
//
// Multi-GPU: `pe_launch -n 8 bin/pe_hip 8192 8192` (or torchrun-style env
// RANK / WORLD_SIZE / LOCAL_RANK).  The RCCL unique id is exchanged through
// a file in $PE_BOOTSTRAP_DIR (set by pe_launch) — no MPI needed.
// --vranks P runs P virtual ranks on one GPU (decomposition testing).
// Output lines follow poisson_mpi_cuda2.cu:1002-1034 (parity) plus the
// L2/max error against the analytic solution the reference never computes.
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <thread>

#include "args.hpp"
#include "pe/device.hpp"

using namespace pe;

static int env_int(const char* a, const char* b, int def) {
  if (const char* v = std::getenv(a)) return std::atoi(v);
  if (const char* v = std::getenv(b)) return std::atoi(v);
  return def;
}

static std::string exchange_uid(int rank, int size) {
  const char* dir = std::getenv("PE_BOOTSTRAP_DIR");
  if (!dir) throw std::runtime_error("multi-rank pe_hip needs PE_BOOTSTRAP_DIR (use pe_launch)");
  const std::string path = std::string(dir) + "/rccl_uid";
  if (rank == 0) {
    const std::string uid = rccl_unique_id();
    const std::string tmp = path + ".tmp";
    std::ofstream(tmp, std::ios::binary).write(uid.data(), std::streamsize(uid.size()));
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot publish rccl uid");
    return uid;
  }
  for (int t = 0; t < 60000; ++t) {
    std::ifstream f(path, std::ios::binary);
    if (f) {
      std::string uid((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
      if (uid.size() == 128) return uid;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  (void)size;
  throw std::runtime_error("timed out waiting for the rccl uid");
}

int main(int argc, char** argv) {
  const auto t_program = std::chrono::steady_clock::now();
  Args args(argc, argv);
  Problem P;
  const auto& pos = args.positional();
  if (pos.size() >= 2) {
    P.M = std::atoi(pos[0].c_str());
    P.N = std::atoi(pos[1].c_str());
  }
  P.tol = args.getd("tol", 1e-6);
  P.max_iter = args.geti("max-iter", -1);
  P.norm = args.get("norm", "weighted") == "unweighted" ? Norm::Unweighted : Norm::Weighted;
  SolveOptions opt;
  opt.init = args.get("init", "zero") == "random" ? Init::Random : Init::Zero;
  opt.seed = uint64_t(args.geti("seed", 1234));
  opt.variant = int(args.geti("variant", 0));
  {
    const std::string a = args.get("algo", "auto");
    opt.algo = a == "classic" ? 1 : a == "fused" ? 2 : a == "two-step" ? 3 : a == "three-step" ? 4 : 0;
  }
  opt.chunk = int(args.geti("chunk", 0));
  opt.use_graph = args.flag("graph") && !args.flag("no-graph");
  opt.timing = args.flag("timing");
  opt.check_tol = !args.flag("no-tol");  // fixed-iteration runs (with --max-iter) for profiling
  opt.checkpoint_path = args.get("checkpoint", "");
  opt.checkpoint_every = args.geti("checkpoint-every", 0);
  opt.resume_path = args.get("resume", "");
  opt.log_every = int(args.geti("log-every", 0));
  const std::string decomp = args.get("decomp", "device");

  const int rank = env_int("PE_RANK", "RANK", 0);
  const int size = env_int("PE_WORLD_SIZE", "WORLD_SIZE", 1);
  const int local = env_int("PE_LOCAL_RANK", "LOCAL_RANK", 0);
  const int vranks = int(args.geti("vranks", 1));

  const int ndev = device_count();
  if (ndev < 1) {
    std::fprintf(stderr, "pe_hip: no HIP device visible\n");
    return 2;
  }
  set_device(local % ndev);
  if (rank == 0 && !args.flag("quiet"))
    std::cout << "HIP + RCCL 2D run with " << size * vranks << " ranks on " << device_name(local % ndev) << "; M="
              << P.M << ", N=" << P.N << std::endl;

  SolveResult r;
  // rank 0's transport diagnostics (first cross-device run: what each
  // self-tested set-up decided, peer access toward every rank)
  std::string diag = "\"halo_push\": \"off: one rank\", \"sums\": \"none\"";
  if (vranks > 1) {
    r = device_solve_group(P, process_grid_from_spec(decomp, vranks, P.M, P.N), opt);
  } else {
    std::unique_ptr<DeviceComm> comm;
    if (size > 1) comm = make_rccl_comm(exchange_uid(rank, size), rank, size);
    // per-iteration sums: the in-sweep P2P sum over xGMI by default (as the
    // torch.distributed launcher, parallel/dist.py); PE_ALLREDUCE=rccl keeps
    // ncclAllReduce.  The P2P set-up self-tests and falls back to RCCL.
    const char* ar = std::getenv("PE_ALLREDUCE");
    if (comm && !(ar && std::string(ar) == "rccl")) comm = make_p2p_allreduce_comm(std::move(comm));
    const ProcessGrid pg = process_grid_from_spec(decomp, size, P.M, P.N);
    const Block blk = decompose(P.M, P.N, pg, rank);
    // T_solver = construction (allocation, tables, placement search) + solve
    // (SolveResult) + teardown (the frees), as the reference's time_solver
    // (poisson_mpi_cuda2.cu:1010-1016)
    auto solver = std::make_unique<DeviceSolver>(P, blk, comm.get(), opt);
    {
      std::string pa;
      for (int v : solver->peer_access()) pa += (pa.empty() ? "" : ", ") + std::to_string(v);
      std::string hc;
      for (const auto& c : solver->halo_candidates()) {
        char b[128];
        std::snprintf(b, sizeof(b), "%s[\"%s\", %.2f]", hc.empty() ? "" : ", ", c.first.c_str(), c.second);
        hc += b;
      }
      diag = "\"p2p_sum_setup\": \"" + p2p_setup_status() + "\", \"halo_push\": \"" + solver->push_status() +
             "\", \"halo_put\": \"" + solver->put_status() + "\", \"halo_path\": \"" + solver->halo_path() +
             "\", \"halo_candidates_us_per_sweep\": [" + hc + "], \"sums\": \"" + solver->xr_status() +
             "\", \"peer_access\": [" + pa + "]";
    }
    r = solver->solve();
    const auto t_free = std::chrono::steady_clock::now();
    solver.reset();
    r.t.solver += std::chrono::duration<double>(std::chrono::steady_clock::now() - t_free).count();
  }
  const double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_program).count();
  if (rank == 0) {
    if (args.flag("json")) {
      std::printf("{\"M\": %d, \"N\": %d, \"ranks\": %d, \"Px\": %d, \"Py\": %d, \"iters\": %lld, \"converged\": %s, "
                  "\"t_solver\": %.6f, \"t_setup\": %.6f, \"t_construct\": %.6f, \"t_iterate\": %.6f, "
                  "\"t_gpu\": %.6f, \"t_dot\": %.6f, \"dot_fused\": %s, \"t_copy\": %.6f, \"t_halo\": %.6f, "
                  "\"t_reduce\": %.6f, \"timer_samples\": %.0f, "
                  "\"iters_per_s\": %.3f, \"l2_err\": %.6e, \"max_err\": %.6e, \"max_outside\": %.6e, \"total\": %.6f, "
                  "\"algo\": \"%s\", \"res_true\": %.6e, \"res_rec\": %.6e, \"res_gap\": %.6e, "
                  "\"b_norm\": %.6e, \"restarts\": %d, \"t_check\": %.6f, %s}\n",
                  P.M, P.N, size * vranks, r.Px, r.Py, (long long)r.iters, r.converged ? "true" : "false", r.t.solver,
                  r.t.setup, r.t.construct, r.t.iterate, r.t.gpu, r.t.dot, r.t.dot_fused ? "true" : "false", r.t.copy,
                  r.t.halo, r.t.reduce, r.t.sampled, r.iters / std::max(1e-12, r.t.iterate), r.l2_err, r.max_err,
                  r.max_outside, total, r.algo.c_str(), r.res_true, r.res_rec, r.res_gap, r.b_norm,
                  r.restarts, r.t.check, diag.c_str());
    } else {
      std::cout << format_result_legacy(P, r, size, "stage4");
      std::printf("   Process grid %dx%d | iters/s ~ %.1f | L2 error in D ~ %.6e | max error in D ~ %.6e\n", r.Px, r.Py,
                  r.iters / std::max(1e-12, r.t.iterate), r.l2_err, r.max_err);
    }
  }
  if (r.nonfinite) {
    std::fprintf(stderr, "pe_hip: a reduced scalar became NaN/Inf at iteration %lld; solve stopped\n",
                 (long long)r.iters);
    return 3;
  }
  return 0;
}
