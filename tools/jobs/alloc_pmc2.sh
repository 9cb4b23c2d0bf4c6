set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/apmc2; mkdir -p $O
export PE_PLACEMENT_TRIES=1
P="python3 $GRAFT_REPO_ROOT/tools/alloc_pmc.py 8"
timeout -k 10 240 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum -d $O/a -o run -- $P > $O/a.log 2>&1
echo EXIT $?
