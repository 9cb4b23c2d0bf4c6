set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rccl2; mkdir -p $O
timeout -k 10 120 ./bin/pe_launch -n 2 ./bin/pe_hip --json 400 600 > $O/pe_launch2.txt 2>&1; echo "pe_launch rc=$?" >> $O/pe_launch2.txt
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 50 --warmup 5 --grid 1024 1024 > $O/bench2.txt 2>&1; echo "bench2 rc=$?" >> $O/bench2.txt
echo EXIT 0
