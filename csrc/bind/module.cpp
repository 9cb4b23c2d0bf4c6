// Python binding of the native core (pybind11).  The package's Python layer
// (poisson_ellipse_openmp_mpi_cuda_amd) adds torch.distributed bootstrap,
// the PyTorch fp64 oracle, the CLI/bench and reporting on top of this.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "../hip/kernels.hpp"
#include "pe/device.hpp"
#include "pe/solver.hpp"

namespace py = pybind11;
using namespace pe;

namespace {

py::dict timers_dict(const Timers& t) {
  py::dict d;
  d["gpu"] = t.gpu;
  d["copy"] = t.copy;
  d["halo"] = t.halo;
  d["reduce"] = t.reduce;
  d["prec"] = t.prec;
  d["dot"] = t.dot;
  d["setup"] = t.setup;
  d["solver"] = t.solver;
  d["iterate"] = t.iterate;
  d["check"] = t.check;
  d["construct"] = t.construct;
  d["sampled"] = t.sampled;
  d["wait"] = t.wait;
  d["dot_fused"] = t.dot_fused;
  return d;
}

py::array_t<double> to_array(std::vector<double>&& v, int64_t rows, int64_t cols) {
  auto* heap = new std::vector<double>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete static_cast<std::vector<double>*>(p); });
  return py::array_t<double>({rows, cols}, {cols * int64_t(sizeof(double)), int64_t(sizeof(double))}, heap->data(),
                             owner);
}

py::dict state_dict(const dev::DevState& s) {
  py::dict d;
  d["red_F"] = py::make_tuple(s.red_F[0], s.red_F[1]);
  d["red_G"] = s.red_G[0];
  d["err"] = py::make_tuple(s.err[0], s.err[1], s.err[2]);
  d["rz_cur"] = s.rz_cur;
  d["alpha"] = s.alpha;
  d["beta"] = s.beta;
  d["last_diff"] = s.last_diff;
  d["iter"] = s.iter;
  d["done"] = s.done;
  d["status"] = s.status;
  d["started"] = s.started;
  d["gprev"] = s.gprev;
  d["fs"] = py::make_tuple(py::make_tuple(s.fs[0][0], s.fs[0][1], s.fs[0][2], s.fs[0][3], s.fs[0][4], s.fs[0][5],
                                          s.fs[0][6]),
                           py::make_tuple(s.fs[1][0], s.fs[1][1], s.fs[1][2], s.fs[1][3], s.fs[1][4], s.fs[1][5],
                                          s.fs[1][6]));
  py::list f2;
  for (int b = 0; b < 2; ++b) {
    py::list v;
    for (int n = 0; n < dev::kNS2; ++n) v.append(s.fs2[b][n]);
    f2.append(py::tuple(v));
  }
  d["fs2"] = py::tuple(f2);
  d["late3"] = s.late3;
  py::list c3;
  for (int n = 0; n < 12; ++n) c3.append(s.sc3[n]);
  d["sc3"] = py::tuple(c3);
  d["wait_s"] = double(s.xr_wait) * 1e-8;
  d["wpar"] = s.wpar;
  d["res"] = py::make_tuple(s.res[0], s.res[1], s.res[2], s.res[3]);
  d["k0"] = s.k0;
  d["fixj"] = s.fixj;
  return d;
}

// Handle to a DeviceComm owned by Python.
struct CommHandle {
  std::unique_ptr<DeviceComm> comm;
};

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "Native core of the MI355X Poisson/fictitious-domain PCG framework (C++ / HIP gfx950 / RCCL)";

  py::enum_<Norm>(m, "Norm").value("Weighted", Norm::Weighted).value("Unweighted", Norm::Unweighted);
  py::enum_<Init>(m, "Init").value("Zero", Init::Zero).value("Random", Init::Random);
  py::enum_<DecompMode>(m, "DecompMode")
      .value("Reference", DecompMode::Reference)
      .value("Aspect", DecompMode::Aspect)
      .value("Rows", DecompMode::Rows)
      .value("Cols", DecompMode::Cols);

  py::class_<Problem>(m, "Problem")
      .def(py::init<>())
      .def_readwrite("A1", &Problem::A1)
      .def_readwrite("B1", &Problem::B1)
      .def_readwrite("A2", &Problem::A2)
      .def_readwrite("B2", &Problem::B2)
      .def_readwrite("F", &Problem::F)
      .def_readwrite("cx", &Problem::cx)
      .def_readwrite("cy", &Problem::cy)
      .def_readwrite("sx", &Problem::sx)
      .def_readwrite("sy", &Problem::sy)
      .def_readwrite("M", &Problem::M)
      .def_readwrite("N", &Problem::N)
      .def_readwrite("tol", &Problem::tol)
      .def_readwrite("max_iter", &Problem::max_iter)
      .def_readwrite("norm", &Problem::norm)
      .def("h1", &Problem::h1)
      .def("h2", &Problem::h2)
      .def("eps", &Problem::eps)
      .def("iter_cap", &Problem::iter_cap)
      .def("u_scale", &Problem::u_scale);

  py::class_<ProcessGrid>(m, "ProcessGrid")
      .def(py::init<>())
      .def_readwrite("Px", &ProcessGrid::Px)
      .def_readwrite("Py", &ProcessGrid::Py);

  py::class_<Block>(m, "Block")
      .def_readonly("rank", &Block::rank)
      .def_readonly("size", &Block::size)
      .def_readonly("Px", &Block::Px)
      .def_readonly("Py", &Block::Py)
      .def_readonly("px", &Block::px)
      .def_readonly("py", &Block::py)
      .def_readonly("i0", &Block::i0)
      .def_readonly("i1", &Block::i1)
      .def_readonly("j0", &Block::j0)
      .def_readonly("j1", &Block::j1)
      .def_readonly("nx", &Block::nx)
      .def_readonly("ny", &Block::ny)
      .def_readonly("pitch", &Block::pitch)
      .def_readonly("rows", &Block::rows)
      .def_readonly("base", &Block::base)
      .def_readonly("alloc", &Block::alloc)
      .def_property_readonly("nbr", [](const Block& b) { return std::vector<int>(b.nbr, b.nbr + 4); })
      .def("__repr__", &describe);

  m.def("choose_process_grid", &choose_process_grid, py::arg("P"), py::arg("M"), py::arg("N"),
        py::arg("mode") = DecompMode::Aspect);
  m.def("choose_process_grid_reference", &choose_process_grid_reference);
  m.def("process_grid_from_spec", &process_grid_from_spec, py::arg("spec"), py::arg("P"), py::arg("M"), py::arg("N"));
  m.def("halo_cost", &halo_cost);
  m.def("decompose", &decompose, py::arg("M"), py::arg("N"), py::arg("pg"), py::arg("rank"), py::arg("align") = 8);

  py::class_<SolveOptions>(m, "SolveOptions")
      .def(py::init<>())
      .def_readwrite("init", &SolveOptions::init)
      .def_readwrite("seed", &SolveOptions::seed)
      .def_readwrite("init_amp", &SolveOptions::init_amp)
      .def_readwrite("threads", &SolveOptions::threads)
      .def_readwrite("log_every", &SolveOptions::log_every)
      .def_readwrite("keep_history", &SolveOptions::keep_history)
      .def_readwrite("compute_error", &SolveOptions::compute_error)
      .def_readwrite("verbose", &SolveOptions::verbose)
      .def_readwrite("chunk", &SolveOptions::chunk)
      .def_readwrite("use_graph", &SolveOptions::use_graph)
      .def_readwrite("timing", &SolveOptions::timing)
      .def_readwrite("check_tol", &SolveOptions::check_tol)
      .def_readwrite("variant", &SolveOptions::variant)
      .def_readwrite("algo", &SolveOptions::algo)
      .def_readwrite("checkpoint_every", &SolveOptions::checkpoint_every)
      .def_readwrite("checkpoint_path", &SolveOptions::checkpoint_path)
      .def_readwrite("resume_path", &SolveOptions::resume_path);

  py::class_<SolveResult>(m, "SolveResult")
      .def_readonly("iters", &SolveResult::iters)
      .def_readonly("converged", &SolveResult::converged)
      .def_readonly("breakdown", &SolveResult::breakdown)
      .def_readonly("nonfinite", &SolveResult::nonfinite)
      .def_readonly("last_diff", &SolveResult::last_diff)
      .def_readonly("zr", &SolveResult::zr)
      .def_readonly("l2_err", &SolveResult::l2_err)
      .def_readonly("max_err", &SolveResult::max_err)
      .def_readonly("max_outside", &SolveResult::max_outside)
      .def_readonly("history", &SolveResult::history)
      .def_readonly("Px", &SolveResult::Px)
      .def_readonly("Py", &SolveResult::Py)
      .def_readonly("backend", &SolveResult::backend)
      .def_readonly("algo", &SolveResult::algo)
      .def_readonly("resident_fallback", &SolveResult::resident_fallback)
      .def_readonly("res_true", &SolveResult::res_true)
      .def_readonly("res_rec", &SolveResult::res_rec)
      .def_readonly("res_gap", &SolveResult::res_gap)
      .def_readonly("b_norm", &SolveResult::b_norm)
      .def_readonly("restarts", &SolveResult::restarts)
      .def_property_readonly("timers", [](const SolveResult& r) { return timers_dict(r.t); });

  m.def("format_result_legacy", &format_result_legacy);
  m.def("p2p_setup_status", []() { return p2p_setup_status(); },
        "the last P2P transport set-up of this process: not attempted / ok / fallback: why");

  // ---- CPU backends ------------------------------------------------------
  m.def(
      "cpu_solve",
      [](const Problem& P, int ranks, DecompMode mode, const SolveOptions& opt, bool return_w) {
        std::vector<double> w;
        SolveResult r;
        {
          py::gil_scoped_release nogil;
          r = cpu_pcg_threads(P, ranks, mode, opt, return_w ? &w : nullptr);
        }
        py::object wa = py::none();
        if (return_w) wa = to_array(std::move(w), P.M - 1, P.N - 1);
        return py::make_tuple(r, wa);
      },
      py::arg("prob"), py::arg("ranks") = 1, py::arg("mode") = DecompMode::Reference, py::arg("opt") = SolveOptions(),
      py::arg("return_w") = false);
  m.def(
      "cpu_solve_grid",
      [](const Problem& P, const ProcessGrid& pg, const SolveOptions& opt, bool return_w) {
        std::vector<double> w;
        SolveResult r;
        {
          py::gil_scoped_release nogil;
          r = cpu_pcg_threads(P, pg, opt, return_w ? &w : nullptr);
        }
        py::object wa = py::none();
        if (return_w) wa = to_array(std::move(w), P.M - 1, P.N - 1);
        return py::make_tuple(r, wa);
      },
      py::arg("prob"), py::arg("grid"), py::arg("opt") = SolveOptions(), py::arg("return_w") = false);

  // One rank of a multi-process CPU run; the transport is Python callbacks
  // (torch.distributed, typically gloo).  exchange_fn receives a list of
  // (dir, peer, send: ndarray, recv: writable ndarray) valid during the call.
  m.def(
      "cpu_solve_rank",
      [](const Problem& P, const Block& blk, py::function reduce_fn, py::function exchange_fn,
         py::function barrier_fn, const SolveOptions& opt, bool return_w) {
        auto reduce = [reduce_fn](double* buf, int n, bool is_max) {
          py::gil_scoped_acquire g;
          py::array_t<double> a({n}, {int64_t(sizeof(double))}, buf, py::none());
          reduce_fn(a, is_max);
        };
        auto exch = [exchange_fn](const std::vector<Exchange>& ex) {
          py::gil_scoped_acquire g;
          py::list items;
          for (const auto& e : ex) {
            py::array_t<double> s({e.count}, {int64_t(sizeof(double))}, const_cast<double*>(e.send), py::none());
            py::array_t<double> r({e.count}, {int64_t(sizeof(double))}, e.recv, py::none());
            items.append(py::make_tuple(e.dir, e.peer, s, r));
          }
          exchange_fn(items);
        };
        auto bar = [barrier_fn]() {
          py::gil_scoped_acquire g;
          barrier_fn();
        };
        CallbackHostComm comm(blk.rank, blk.size, reduce, exch, bar);
        std::vector<double> w;
        SolveResult r;
        {
          py::gil_scoped_release nogil;
          r = cpu_pcg(P, blk, comm, opt, return_w ? &w : nullptr);
        }
        py::object wa = py::none();
        if (return_w) wa = to_array(std::move(w), blk.nx, blk.ny);
        return py::make_tuple(r, wa);
      },
      py::arg("prob"), py::arg("block"), py::arg("reduce_fn"), py::arg("exchange_fn"), py::arg("barrier_fn"),
      py::arg("opt") = SolveOptions(), py::arg("return_w") = false);

  m.def("host_coefficients", [](const Problem& P, const Block& blk) {
    std::vector<double> a, b;
    std::vector<int> c;
    host_coefficients(P, blk, a, b, c);
    const int64_t R = blk.nx + 2, C = blk.ny + 2;
    auto* heap = new std::vector<int>(std::move(c));
    py::capsule owner(heap, [](void* p) { delete static_cast<std::vector<int>*>(p); });
    py::array_t<int> ca({R, C}, {C * int64_t(sizeof(int)), int64_t(sizeof(int))}, heap->data(), owner);
    return py::make_tuple(to_array(std::move(a), R, C), to_array(std::move(b), R, C), ca);
  });

  // ---- device (HIP / RCCL) ----------------------------------------------
  m.def("device_count", &device_count);
  m.def("set_device", &set_device);
  m.def("device_name", &device_name);
  m.def("current_device", &current_device);
  m.def("device_pci_bus_id", &device_pci_bus_id, py::arg("dev"));
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });

  py::class_<CommHandle>(m, "DeviceComm")
      .def_property_readonly("rank", [](const CommHandle& h) { return h.comm->rank(); })
      .def_property_readonly("size", [](const CommHandle& h) { return h.comm->size(); })
      .def_property_readonly("name", [](const CommHandle& h) { return h.comm->name(); })
      .def(
          "bench_allreduce",
          [](CommHandle& h, int n, int iters) {
            // stream-ordered latency of the in-place sum of n doubles (collective)
            py::gil_scoped_release nogil;
            double* d = nullptr;
            hipStream_t s = nullptr;
            hipEvent_t e0, e1;
            PE_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            PE_HIP_CHECK(hipMalloc(&d, sizeof(double) * std::max(1, n)));
            PE_HIP_CHECK(hipMemsetAsync(d, 0, sizeof(double) * std::max(1, n), s));
            PE_HIP_CHECK(hipEventCreate(&e0));
            PE_HIP_CHECK(hipEventCreate(&e1));
            for (int i = 0; i < 5; ++i) h.comm->allreduce_sum(d, n, s);
            h.comm->barrier(s);
            PE_HIP_CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i) h.comm->allreduce_sum(d, n, s);
            PE_HIP_CHECK(hipEventRecord(e1, s));
            PE_HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            PE_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            (void)hipFree(d);
            (void)hipStreamDestroy(s);
            return 1e3 * double(ms) / std::max(1, iters);
          },
          py::arg("n") = 7, py::arg("iters") = 1000,
          "Microseconds per in-place allreduce_sum of n doubles (call on every rank).");
  m.def(
      "make_rccl_comm",
      [](py::bytes uid, int rank, int size) {
        auto h = std::make_unique<CommHandle>();
        std::string s = uid;
        py::gil_scoped_release nogil;
        h->comm = make_rccl_comm(s, rank, size);
        return h;
      },
      py::arg("uid"), py::arg("rank"), py::arg("size"));
  m.def(
      "make_delay_comm",
      [](int size, double exchange_us, double allreduce_us, bool loopback) {
        auto h = std::make_unique<CommHandle>();
        h->comm = make_delay_comm(size, exchange_us, allreduce_us, loopback);
        return h;
      },
      py::arg("size"), py::arg("exchange_us"), py::arg("allreduce_us"), py::arg("loopback") = false);
  m.def(
      "make_host_staged_comm",
      [](int rank, int size, py::function reduce_fn, py::function exchange_fn, py::function barrier_fn) {
        auto reduce = [reduce_fn](double* buf, int n, bool is_max) {
          py::gil_scoped_acquire g;
          py::array_t<double> a({n}, {int64_t(sizeof(double))}, buf, py::none());
          reduce_fn(a, is_max);
        };
        auto exch = [exchange_fn](const std::vector<Exchange>& ex) {
          py::gil_scoped_acquire g;
          py::list items;
          for (const auto& e : ex) {
            py::array_t<double> s({e.count}, {int64_t(sizeof(double))}, const_cast<double*>(e.send), py::none());
            py::array_t<double> r({e.count}, {int64_t(sizeof(double))}, e.recv, py::none());
            items.append(py::make_tuple(e.dir, e.peer, s, r));
          }
          exchange_fn(items);
        };
        auto bar = [barrier_fn]() {
          py::gil_scoped_acquire g;
          barrier_fn();
        };
        auto h = std::make_unique<CommHandle>();
        h->comm = make_callback_device_comm(rank, size, reduce, exch, bar);
        return h;
      },
      py::arg("rank"), py::arg("size"), py::arg("reduce_fn"), py::arg("exchange_fn"), py::arg("barrier_fn"));
  m.def(
      "use_p2p_allreduce",
      [](CommHandle& h) {
        py::gil_scoped_release nogil;
        h.comm = make_p2p_allreduce_comm(std::move(h.comm));
      },
      py::arg("comm"),
      "Switch the per-iteration sums of this communicator to the one-shot P2P allreduce (collective: call on "
      "every rank).");
  m.def(
      "make_rccl_comm_from_handle",
      [](uintptr_t handle) {
        auto h = std::make_unique<CommHandle>();
        h->comm = make_rccl_comm_from_handle(reinterpret_cast<void*>(handle));
        return h;
      },
      py::arg("nccl_comm_ptr"));

  py::class_<DeviceSolver>(m, "DeviceSolver")
      .def(py::init([](const Problem& P, const Block& blk, CommHandle* comm, const SolveOptions& opt) {
             return std::make_unique<DeviceSolver>(P, blk, comm ? comm->comm.get() : nullptr, opt);
           }),
           py::arg("prob"), py::arg("block"), py::arg("comm") = nullptr, py::arg("opt") = SolveOptions(),
           py::keep_alive<1, 4>())
      .def("solve",
           [](DeviceSolver& s) {
             py::gil_scoped_release nogil;
             return s.solve();
           })
      .def("reset", [](DeviceSolver& s) {
        py::gil_scoped_release nogil;
        s.reset();
        s.synchronize();
      })
      .def("run_iterations",
           [](DeviceSolver& s, int64_t n, bool g) {
             py::gil_scoped_release nogil;
             s.run_iterations(n, g);
           },
           py::arg("iters"), py::arg("use_graph") = true)
      .def("set_check_tol", &DeviceSolver::set_check_tol, py::arg("on"))
      .def("set_init", &DeviceSolver::set_init, py::arg("init"), py::arg("seed") = 1234, py::arg("amp") = 0.05)
      .def("relayout", &DeviceSolver::relayout, py::arg("ti"), py::arg("order") = -1)
      .def("prepare_graphs",
           [](DeviceSolver& s, int64_t n) {
             py::gil_scoped_release nogil;
             s.prepare_graphs(n);
           },
           py::arg("iters"))
      .def("time_iterations",
           [](DeviceSolver& s, int64_t n, bool g) {
             py::gil_scoped_release nogil;
             return s.time_iterations(n, g);
           },
           py::arg("iters"), py::arg("use_graph") = true)
      .def("synchronize", [](DeviceSolver& s) {
        py::gil_scoped_release nogil;
        s.synchronize();
      })
      .def("state",
           [](DeviceSolver& s) {
             dev::DevState st;
             s.read_state(&st);
             return state_dict(st);
           })
      .def("w",
           [](DeviceSolver& s) {
             const Block& b = s.block();
             std::vector<double> v(size_t(b.nx * b.ny));
             s.copy_w(v.data());
             return to_array(std::move(v), b.nx, b.ny);
           })
      .def("field",
           [](DeviceSolver& s, int which) {
             std::vector<double> v(size_t(s.field_rows() * s.field_cols()));
             s.copy_field(which, v.data());
             return to_array(std::move(v), s.field_rows(), s.field_cols());
           })
      .def_property_readonly("chunk", &DeviceSolver::chunk)
      .def_property_readonly("fused", &DeviceSolver::fused)
      .def_property_readonly("two_step", &DeviceSolver::two_step, "several iterations per sweep (fused2.hip / fused3.hip)")
      .def_property_readonly("sweep_steps", &DeviceSolver::sweep_steps, "iterations per sweep launch (1, 2, 3)")
      .def_property_readonly("resident", &DeviceSolver::resident)
      .def_property_readonly("resident_fallback", &DeviceSolver::resident_fallback)
      .def_property_readonly("layout_cuts", &DeviceSolver::layout_cuts)
      .def_property_readonly("layout_name", &DeviceSolver::layout_name, "static item layout: lpt / fill / equal")
      .def_property_readonly(
          "layout_entries",
          [](const DeviceSolver& s) {
            // (first row, rows, strip, flags) per list position; rows 0: an empty position
            std::vector<std::tuple<int, int, int, int>> v;
            for (const int2& e : s.layout_entries())
              v.emplace_back(e.x & dev::kRowMask3, e.y >> 20, e.y & 0xFFFFF, e.x & ~dev::kRowMask3);
            return v;
          },
          "the static item list: (first row, rows, strip, flags: kBandBit | kUniBit)")
      .def_property_readonly("layout_waves", [](DeviceSolver& s) { return s.params().lwaves; })
      .def_property_readonly("strips", [](DeviceSolver& s) { return s.params().nstrips; }, "wave strips across the block")
      .def_property_readonly("layout_boundary", &DeviceSolver::layout_boundary,
                             "overlap: list positions 0 .. n-1 hold the boundary items (0: no overlap)")
      .def_property_readonly("peer_access", &DeviceSolver::peer_access,
                             "hipDeviceCanAccessPeer toward each rank's device (1/0; -1 same device)")
      .def_property_readonly("push_status", &DeviceSolver::push_status, "halo push: on / off: why / fallback: why")
      .def_property_readonly("xr_status", &DeviceSolver::xr_status, "transport of the per-sweep sums")
      .def_property_readonly("overlap", &DeviceSolver::overlap)
      .def_property_readonly("halo_push", &DeviceSolver::halo_push,
                             "halo rows pushed by the sweep over xGMI (no exchange call; graph-capturable)")
      .def_property_readonly("halo_put", &DeviceSolver::halo_put,
                             "halo phases exchanged by the peer-put kernel (p2p.hip kPut) instead of the comm")
      .def_property_readonly("halo_path", &DeviceSolver::halo_path,
                             "the multi-rank halo path chosen at construction (exchange / put / push [+overlap])")
      .def_property_readonly("halo_candidates", &DeviceSolver::halo_candidates,
                             "[(path, µs per sweep)] as timed by the construction's halo-path choice (max over ranks)")
      .def_property_readonly("graphs_usable", &DeviceSolver::graphs_usable)
      .def("set_halo_path", &DeviceSolver::set_halo_path, py::arg("path"), py::arg("overlap"),
           "probe: switch to another halo path candidate (exchange / put / push, overlap)")
      .def("time_halo_path", &DeviceSolver::time_halo_path, py::arg("sweeps") = 4, py::arg("warm") = 2,
           py::arg("from_reset") = true, "probe: ms per sweep of the current halo path")
      .def_property_readonly("put_status", &DeviceSolver::put_status, "peer put: available / off: why / fallback: why")
      .def("save_checkpoint", &DeviceSolver::save_checkpoint, py::arg("path"))
      .def("load_checkpoint", &DeviceSolver::load_checkpoint, py::arg("path"))
      .def_property_readonly("fields_address", &DeviceSolver::fields_address)
      .def_property_readonly("placement_ms", &DeviceSolver::placement_ms)
      .def_property_readonly("placement_choice", &DeviceSolver::placement_choice)
      .def_property_readonly("placement_s", &DeviceSolver::placement_seconds)
      .def_property_readonly("placement_job_ms", &DeviceSolver::placement_job_ms)
      .def_property_readonly("construct_s", &DeviceSolver::construct_seconds)
      .def_property_readonly("exchange_us", &DeviceSolver::exchange_us)
      .def_property_readonly("ti_tuning_ms", &DeviceSolver::ti_tuning_ms)
      .def_property_readonly("ti_tuning_rows", &DeviceSolver::ti_tuning_rows)
      .def_property_readonly("layout_load", &DeviceSolver::layout_load)
      .def_property_readonly("ti", [](DeviceSolver& s) { return s.params().ti; })
      .def_property_readonly("order", [](DeviceSolver& s) { return s.params().order; })
      .def_property_readonly("xr", [](DeviceSolver& s) { return s.params().xr.peers != nullptr; },
                             "True when the sweep sums its scalars over ranks itself (P2P transport)")
      .def_property_readonly("nitems", [](DeviceSolver& s) { return s.params().nslots; })
      .def_property_readonly("stamp_waves",
                             [](DeviceSolver& s) { return dev::kWPB * std::max(s.params().nblocks, s.params().nblocks0); })
      .def("stamps",
           [](DeviceSolver& s) {
             std::vector<unsigned long long> v = s.stamps();
             py::array_t<unsigned long long> a(py::ssize_t(v.size()));
             if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), sizeof(unsigned long long) * v.size());
             return a;
           },
           "PE_STAMPS=1 diagnostic timeline of the last sweep (tools/stamp_probe.py).")
      .def("clear_stamps", &DeviceSolver::clear_stamps)
      .def_property_readonly("blocks", [](DeviceSolver& s) { return dev::grid_blocks(s.params()); })
      .def_property_readonly("block", &DeviceSolver::block);

  m.def(
      "device_solve_group",
      [](const Problem& P, int ranks, DecompMode mode, const SolveOptions& opt, bool return_w) {
        std::vector<double> w;
        SolveResult r;
        {
          py::gil_scoped_release nogil;
          r = device_solve_group(P, ranks, mode, opt, return_w ? &w : nullptr);
        }
        py::object wa = py::none();
        if (return_w) wa = to_array(std::move(w), P.M - 1, P.N - 1);
        return py::make_tuple(r, wa);
      },
      py::arg("prob"), py::arg("ranks"), py::arg("mode") = DecompMode::Aspect, py::arg("opt") = SolveOptions(),
      py::arg("return_w") = false);

  m.def(
      "device_solve_group_grid",
      [](const Problem& P, const ProcessGrid& pg, const SolveOptions& opt, bool return_w) {
        std::vector<double> w;
        SolveResult r;
        {
          py::gil_scoped_release nogil;
          r = device_solve_group(P, pg, opt, return_w ? &w : nullptr);
        }
        py::object wa = py::none();
        if (return_w) wa = to_array(std::move(w), P.M - 1, P.N - 1);
        return py::make_tuple(r, wa);
      },
      py::arg("prob"), py::arg("grid"), py::arg("opt") = SolveOptions(), py::arg("return_w") = false);

  // Single-shot device ops for numerics tests: `p` is a full local field
  // (rows × pitch, halo included); returns arrays of the same shape.
  m.def("device_apply_A", [](const Problem& P, const Block& blk, py::array_t<double, py::array::c_style> p) {
    if (p.size() != blk.rows * blk.pitch) throw std::invalid_argument("p must be rows x pitch");
    SolveOptions opt;
    opt.algo = 1;  // classic layout: p is rows × pitch of the block
    DeviceSolver s(P, blk, nullptr, opt);
    const size_t bytes = sizeof(double) * blk.rows * blk.pitch;
    double *dp = nullptr, *dA = nullptr;
    PE_HIP_CHECK(hipMalloc(&dp, bytes));
    PE_HIP_CHECK(hipMalloc(&dA, bytes));
    // everything on the solver's (non-blocking) stream: a null-stream memset
    // is not ordered with it
    PE_HIP_CHECK(hipMemcpyAsync(dp, p.data(), bytes, hipMemcpyHostToDevice, s.stream()));
    PE_HIP_CHECK(hipMemsetAsync(dA, 0, bytes, s.stream()));
    dev::launch_apply_A(s.params(), dp, dA, s.stream());
    std::vector<double> out(blk.rows * blk.pitch);
    PE_HIP_CHECK(hipStreamSynchronize(s.stream()));
    PE_HIP_CHECK(hipMemcpy(out.data(), dA, bytes, hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipFree(dp));
    PE_HIP_CHECK(hipFree(dA));
    return to_array(std::move(out), blk.rows, blk.pitch);
  });
  m.def("device_coefficients", [](const Problem& P, const Block& blk) {
    SolveOptions opt;
    opt.algo = 1;
    DeviceSolver s(P, blk, nullptr, opt);
    const size_t n = size_t(blk.rows * blk.pitch), bytes = sizeof(double) * n;
    double* d = nullptr;
    PE_HIP_CHECK(hipMalloc(&d, 3 * bytes));
    PE_HIP_CHECK(hipMemsetAsync(d, 0, 3 * bytes, s.stream()));  // ordered with the kernel (non-blocking stream)
    dev::launch_coef(s.params(), d, d + n, d + 2 * n, s.stream());
    PE_HIP_CHECK(hipStreamSynchronize(s.stream()));
    std::vector<double> a(n), b(n), D(n);
    PE_HIP_CHECK(hipMemcpy(a.data(), d, bytes, hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipMemcpy(b.data(), d + n, bytes, hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipMemcpy(D.data(), d + 2 * n, bytes, hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipFree(d));
    return py::make_tuple(to_array(std::move(a), blk.rows, blk.pitch), to_array(std::move(b), blk.rows, blk.pitch),
                          to_array(std::move(D), blk.rows, blk.pitch));
  });
  m.def("device_coefficients_fast", [](const Problem& P, const Block& blk) {
    SolveOptions opt;
    opt.algo = 2;  // single-sweep tables (row classes / chord tables past the halo)
    DeviceSolver s(P, blk, nullptr, opt);
    const int64_t rows = blk.nx + 2, cols = blk.ny + 2;
    const size_t n = size_t(rows * cols), bytes = sizeof(double) * n;
    double* d = nullptr;
    PE_HIP_CHECK(hipMalloc(&d, 3 * bytes));
    dev::launch_coef_fast(s.params(), d, d + n, d + 2 * n, s.stream());
    PE_HIP_CHECK(hipStreamSynchronize(s.stream()));
    std::vector<double> a(n), b(n), di(n);
    PE_HIP_CHECK(hipMemcpy(a.data(), d, bytes, hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipMemcpy(b.data(), d + n, bytes, hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipMemcpy(di.data(), d + 2 * n, bytes, hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipFree(d));
    return py::make_tuple(to_array(std::move(a), rows, cols), to_array(std::move(b), rows, cols),
                          to_array(std::move(di), rows, cols));
  });
}
