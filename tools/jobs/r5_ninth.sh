# Round 5, ninth GPU call: stamped sweeps repeated in one process — is a
# slow item / wave slow again in the next sweep (persistence correlations,
# per-XCD mean exits)? — and the last block's epilogue broken down (block
# reduce, publish, ticket, partials summed, finalize) at the 8-rank slab,
# the 4x2 block, 2048^2 and 8192^2 on 1 GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ninth; mkdir -p $O
cd $R
PROBE_REPEAT=6 PROBE_CFG=8:device,8:4x2 timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps_mid.txt 2>&1 || { tail -20 $O/stamps_mid.txt; exit 1; }
PROBE_REPEAT=6 PROBE_GRID=2048x2048 PROBE_CFG=1:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps2048.txt 2>&1 || { tail -20 $O/stamps2048.txt; exit 1; }
PROBE_REPEAT=4 PROBE_CFG=1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps8192.txt 2>&1 || { tail -20 $O/stamps8192.txt; exit 1; }
grep -h -E "^P=|persistence|sweeps [0-9]|averaged|by XCD|last block|launch timeline|gap after|walk entry|first item start|last wave exit|busy fraction|tail" $O/stamps_mid.txt $O/stamps2048.txt $O/stamps8192.txt
echo EXIT 0
