# Construction-phase breakdown (PE_CTOR_TRACE=1) of the published grids:
# fresh process (bin/pe_hip) and a warm second solve in one Python process.
cd $GRAFT_REPO_ROOT
O=gpurun_out/ctor; mkdir -p $O
for g in "800 1200" "1600 2400" "2400 3200" "8192 8192"; do
  echo "== bin/pe_hip $g"
  PE_CTOR_TRACE=1 timeout -k 10 60 bin/pe_hip --json $g 2>&1 | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('  t_solver %.4f setup %.4f construct %.4f iterate %.4f copy %.4f' % (d['t_solver'], d['t_setup'], d['t_construct'], d['t_iterate'], d['t_copy']))
    else: print(' ', l.rstrip())
" || exit 1
done
echo "== warm (second solver in one process)"
PE_CTOR_TRACE=1 timeout -k 10 90 python -u -c "
import sys; sys.path.insert(0,'.')
import poisson_ellipse_openmp_mpi_cuda_amd as pe
for g in [(800,1200),(800,1200),(1600,2400),(2400,3200)]:
    r = pe.solve(pe.EllipseProblem(*g), backend='hip')
    t = r.timers
    print(g, 'iters', r.iters, 'solver %.4f setup %.4f construct %.4f iterate %.4f' % (t['solver'], t['setup'], t['construct'], t['iterate']), flush=True)
" 2>&1 | grep -v amdgpu.ids
