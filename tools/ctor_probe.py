import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, native
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D
nat = native(); nat.set_device(0)
for M, N in [(2400, 3200), (4096, 4096), (2400, 3200)]:
    for tune in ("1", "0"):
        os.environ["PE_TI_TUNE"] = tune
        t0 = time.perf_counter()
        s = nat.DeviceSolver(EllipseProblem(M, N).to_native(), D.block(M, N, 1, 0), None, nat.SolveOptions())
        t1 = time.perf_counter()
        print(f"{M}x{N} tune={tune}: ctor {t1-t0:.3f} s, construct_s {s.construct_s:.3f}, placement_s {s.placement_s:.3f}, "
              f"placement {[round(x,3) for x in s.placement_ms]}, ti {s.ti}, tuning {[round(x,4) for x in s.ti_tuning_ms]}", flush=True)
        del s
