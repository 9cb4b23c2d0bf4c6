# Round 5, eighth GPU call: (1) rehearsal of the driver's 8-GPU bench at the
# real config — 8 processes on the one GPU, 8192^2, row slabs with the
# in-sweep halo push and P2P sums (host-staged base transport: RCCL refuses
# two ranks on one device); the 4x2 split through the exchange + overlap;
# (2) HEAD 1-GPU bench + per-rank probes after the band cost change;
# (3) 2048^2 full solve (BASELINE config 2) -> profiles/r5_rehearsal.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5eighth; mkdir -p $O
cd $R
P=29517
PE_COMM=host PE_ALLREDUCE=p2p PE_P2P_TIMEOUT_S=60 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 8 --steps 20 --warmup 5 --no-random-solve > $O/r8.json 2> $O/r8.err || { tail -20 $O/r8.err; exit 1; }
PE_COMM=host PE_ALLREDUCE=p2p PE_P2P_TIMEOUT_S=60 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((P+1)) bench.py --gpus 8 --steps 20 --warmup 5 --decomp 4x2 --no-random-solve > $O/r8x42.json 2> $O/r8x42.err || { tail -20 $O/r8x42.err; exit 1; }
python3 -c "
import json
for n in ('r8','r8x42'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); c=d['config']
    print(n, 'valid', d['valid'], 'value', round(d['value'],1), 'iters', d.get('iters_converged'), 'conv', d.get('converged'), 'l2', d.get('l2_err'), 'decomp', c['decomposition'], 'halo', c['halo'], 'allreduce', c['allreduce'], 'overlap', c['overlap'], 'ex_us', c.get('exchange_us_measured'))
    for r in c['ranks'][:3]: print('   rank', r['rank'], r.get('halo_push'), r.get('sums'), r.get('p2p_sum_setup'), r.get('peer_access'))"
for i in 1 2; do timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/b$i.json 2> $O/b$i.err || exit 1; done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --grid 2048 2048 > $O/b2048.json 2> $O/b2048.err || exit 1
python3 -c "
import json
for n in ('b1','b2','b2048'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print(n, round(d['value'],1), d.get('iters_converged'), 't_solver', d.get('t_solver_s'), 't_iterate', d.get('t_iterate_s'), 't_check', d.get('t_check_s'), d['config']['ranks'][0]['pci_bus_id'])"
PROBE_CFG=8:device,8:4x2,4:device,2:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe.txt 2>&1 || exit 1
grep -h "us/iter" $O/probe.txt
PROBE_CFG=8:4x2 PROBE_GRAPH=0 timeout -k 10 120 python -u tools/overlap_probe.py 15 8 > $O/overlap.txt 2>&1 || exit 1
grep -h "us/iter" $O/overlap.txt
echo EXIT 0
