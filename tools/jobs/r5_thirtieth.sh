# Round 5, thirtieth GPU call: final driver-shaped checks at HEAD — smoke(),
# the default 1-GPU bench (as the driver runs it), the 8-rank rehearsal of the
# 8-GPU bench at the real config (8 processes on the one GPU, host-staged base
# transport, in-sweep P2P sums + halo push), and the 4x2 rehearsal.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtieth; mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 200 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json
P=29617
PE_COMM=host PE_ALLREDUCE=p2p PE_P2P_TIMEOUT_S=60 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 8 --steps 20 --warmup 5 --no-random-solve > $O/r8.json 2> $O/r8.err || { tail -20 $O/r8.err; exit 1; }
PE_COMM=host PE_ALLREDUCE=p2p PE_P2P_TIMEOUT_S=60 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((P+1)) bench.py --gpus 8 --steps 20 --warmup 5 --decomp 4x2 --no-random-solve > $O/r8x42.json 2> $O/r8x42.err || { tail -20 $O/r8x42.err; exit 1; }
python3 -c "
import json
for n in ('r8','r8x42'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); c=d['config']
    print(n, 'valid', d['valid'], 'value', round(d['value'],1), 'iters', d.get('iters_converged'), 'conv', d.get('converged'), 'l2', d.get('l2_err'), 'halo', c['halo'], 'allreduce', c['allreduce'], 'overlap', c['overlap'])
    for r in c['ranks'][:2]: print('   rank', r['rank'], r.get('halo_push'), r.get('sums'), r.get('p2p_sum_setup'))"
echo EXIT 0
