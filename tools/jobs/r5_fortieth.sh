# Round 5, fortieth GPU call: the row slab's two halo paths on one GPU — the
# push kernel (PE_PUSH_LOOPBACK=1) against the exchange path (PE_HALO=exchange:
# plain sweep + pack / exchange / unpack) at 15 / 8 us exchange / sum delays,
# with and without the overlap (tools/overlap_probe.py), 8192^2 8 and 4 ranks.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fortieth; mkdir -p $O
cd $R
PE_PUSH_LOOPBACK=1 PROBE_CFG=8:device,4:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/push loopback /"
PE_HALO=exchange PROBE_CFG=8:device,4:device PROBE_GRAPH=0 timeout -k 10 300 python -u tools/overlap_probe.py 15 8 > $O/overlap.txt 2>&1 || { tail -20 $O/overlap.txt; exit 1; }
grep -h "us/iter" $O/overlap.txt | sed "s/^/exchange /"
echo EXIT 0
