for i in 1 2; do PE_CTOR_TRACE=1 timeout -k 5 60 bin/pe_hip --json 800 1200 2>&1 | grep -v amdgpu.ids | cut -c1-150; done
PE_CTOR_TRACE=1 timeout -k 5 60 python -c "
import sys; sys.path.insert(0,'.')
import poisson_ellipse_openmp_mpi_cuda_amd as pe
for i in range(2): print(pe.solve(pe.EllipseProblem(800,1200), backend='hip').timers['solver'])
" 2>&1 | grep -v amdgpu.ids
