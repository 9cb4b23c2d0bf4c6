# Round 2: HBM ceiling (bin/roofline) and the 16384² pin (classic vs single sweep).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2_pin; mkdir -p $O
timeout -k 10 300 bin/roofline > $O/roofline.txt 2>&1 || { cat $O/roofline.txt; exit 1; }
cat $O/roofline.txt
timeout -k 10 150 bin/pe_hip --json --algo fused 16384 16384 > $O/f16k.json 2>&1 || exit 1
tail -1 $O/f16k.json
timeout -k 10 240 bin/pe_hip --json --algo classic 16384 16384 > $O/c16k.json 2>&1 || exit 1
tail -1 $O/c16k.json
echo EXIT 0
