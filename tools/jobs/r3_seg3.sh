# Segment layout (PE_SEGMENTS=1: one tall equal-cost item per wave, the 12
# pipeline-fill rows paid once per segment) vs LPT items, three-step sweep, on
# the row-slab blocks of 8192^2 and the mid single-GPU grids (tools/layout_probe.py,
# one memory placement per block).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
run() {  # grid P spec cfgs
  echo "== $1 P=$2"
  PROBE_GRID=$1 PROBE_P=$2 PROBE_SPEC=$3 PROBE_ITERS=600 PROBE_ROUNDS=2 PROBE_CFGS="$4" \
    timeout -k 10 200 python3 -u tools/layout_probe.py || exit 1
}
run 8192x8192 8 rows "32;40;32 PE_SEGMENTS=1;32 PE_SEGMENTS=1 PE_GEN_COST=1.5;32 PE_SEGMENTS=1 PE_GEN_COST=3"
run 8192x8192 4 rows "64;48;32 PE_SEGMENTS=1;32 PE_SEGMENTS=1 PE_GEN_COST=3"
run 8192x8192 2 rows "64;80;32 PE_SEGMENTS=1"
run 2400x3200 1 device "32;48;32 PE_SEGMENTS=1"
run 4096x4096 1 device "64;32 PE_SEGMENTS=1"
echo EXIT 0
