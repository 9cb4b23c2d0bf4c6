set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "gfx|Marketing" > gpurun_out/first_info.txt || true
timeout -k 10 60 ./bin/pe_hip 40 40 > gpurun_out/first_40.txt 2>&1 && \
timeout -k 10 120 ./bin/pe_hip 800 1200 > gpurun_out/first_800.txt 2>&1 && \
timeout -k 10 120 ./bin/pe_hip 2048 2048 > gpurun_out/first_2048.txt 2>&1 && \
timeout -k 10 120 ./bin/pe_hip --vranks 4 800 1200 > gpurun_out/first_v4.txt 2>&1 && \
timeout -k 10 120 ./bin/pe_hip --timing 2048 2048 > gpurun_out/first_2048t.txt 2>&1 && \
timeout -k 10 300 ./bin/pe_hip 8192 8192 > gpurun_out/first_8192.txt 2>&1 && \
timeout -k 10 120 python -c "
import torch, importlib.util
spec = importlib.util.spec_from_file_location('_native', 'poisson_ellipse_openmp_mpi_cuda_amd/_native.cpython-310-x86_64-linux-gnu.so')
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
print('torch', torch.__version__, torch.cuda.is_available(), m.device_count(), m.device_name(0))
P = m.Problem(); P.M=800; P.N=1200
b = m.decompose(P.M, P.N, m.choose_process_grid(1, P.M, P.N), 0)
s = m.DeviceSolver(P, b)
r = s.solve(); print(r.iters, r.l2_err, r.timers)
x = torch.zeros(10, device='cuda'); print(x.sum().item())
" > gpurun_out/first_py.txt 2>&1
echo EXIT $?
