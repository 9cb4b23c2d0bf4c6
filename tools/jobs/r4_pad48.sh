# Row padding vs rows per item at 8192^2, aligned 48-column strips: one solver
# per configuration (tools/block_probe.py P=1, each with its own placement
# search) -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PROBE_CFG=1:device PROBE_ENV="PE_TI=104;PE_TI=104 PE_PAD=64;PE_TI=104 PE_PAD=256;PE_TI=112;PE_TI=112 PE_PAD=64;PE_TI=112 PE_PAD=256;PE_TI=80;PE_TI=80 PE_PAD=64;PE_TI=104;PE_TI=112" timeout -k 10 400 python3 -u tools/block_probe.py > $O/r4_pad48.txt 2>&1 || { tail $O/r4_pad48.txt; exit 1; }
cat $O/r4_pad48.txt
echo EXIT 0
