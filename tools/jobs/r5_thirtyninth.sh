# Round 5, thirty-ninth GPU call: the push / P2P / multi-process tests with the
# push's plain layout (the new default), then the 8-rank rehearsal.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtyninth; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_multigpu.py tests/test_gpu.py tests/test_residual.py tests/test_layout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
PE_COMM=host PE_ALLREDUCE=p2p PE_P2P_TIMEOUT_S=60 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29717 bench.py --gpus 8 --steps 20 --warmup 5 --no-random-solve > $O/r8.json 2> $O/r8.err || { tail -20 $O/r8.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/r8.json').read().strip().splitlines()[-1]); c=d['config']
print('r8 valid', d['valid'], 'iters', d.get('iters_converged'), 'conv', d.get('converged'), 'l2', d.get('l2_err'), 'halo', c['halo'], 'allreduce', c['allreduce'])"
echo EXIT 0
