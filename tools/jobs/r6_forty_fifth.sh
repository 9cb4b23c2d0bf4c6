# Round 6, forty-fifth GPU call: three-step vs two-step sweep on the 8- and
# 4-rank slab blocks and the 4x2 block of 8192² (tools/block_probe.py,
# timing-only transport, tuned rows per item): does the two-step sweep's
# shorter pipeline fill pay on mid-size blocks?
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fortyfifth; mkdir -p $O
cd $R
PROBE_CFG=8:rows,4:rows,8:4x2 PROBE_ENV="PE_STEPS=3;PE_STEPS=2;PE_STEPS=3;PE_STEPS=2" PROBE_ITERS=300 timeout -k 10 400 python3 -u tools/block_probe.py > $O/b.txt 2>&1 || { tail -20 $O/b.txt; exit 1; }
grep -v amdgpu.ids $O/b.txt | cut -c1-200
echo EXIT 0
