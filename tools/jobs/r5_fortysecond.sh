# Round 5, forty-second GPU call: final rehearsal of the driver's 8-GPU bench
# at the real config with the new default halo path (row slabs exchange,
# in-sweep P2P sums; 8 processes on the one GPU, host-staged base transport),
# the 2-rank default, smoke() and the 1-GPU bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fortysecond; mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
P=29817
for n in 8 2; do
  PE_COMM=host PE_ALLREDUCE=p2p PE_P2P_TIMEOUT_S=60 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((P+n)) bench.py --gpus $n --steps 20 --warmup 5 --no-random-solve > $O/r$n.json 2> $O/r$n.err || { tail -20 $O/r$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/r$n.json').read().strip().splitlines()[-1]); c=d['config']
print('r$n valid', d['valid'], 'iters', d.get('iters_converged'), 'conv', d.get('converged'), 'l2', d.get('l2_err'), 'halo', c['halo'], 'allreduce', c['allreduce'], 'overlap', c['overlap'])
for r in c['ranks'][:2]: print('   rank', r['rank'], r.get('halo_push'), r.get('sums'))"
done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/b1.json 2> $O/b1.err || exit 1
python3 -c "
import json
d=json.loads(open('$O/b1.json').read().strip().splitlines()[-1]); print('b1', round(d['value'],1), d.get('iters_converged'), d['config']['ranks'][0]['pci_bus_id'])"
echo EXIT 0
