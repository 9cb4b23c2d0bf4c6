# Round 2: the reference's CPU stages 0-3 (bin/pe_cpu) on the GPU box's CPU share
# (16 cores for one GPU): stage0 grid loop, sequential, OpenMP sweep, thread-ranks, hybrid.
set -o pipefail
cd $GRAFT_REPO_ROOT
echo "# nproc $(nproc), OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}"
echo "## stage0"; timeout -k 10 60 bin/pe_cpu --stage stage0 | grep "Iter=" || exit 1
echo "## stage0 sequential"; for g in "400 600" "800 1200"; do timeout -k 10 120 bin/pe_cpu --backend serial $g | grep "Iter=" || exit 1; done
echo "## stage1 OpenMP"; timeout -k 10 120 bin/pe_cpu --backend omp --threads-sweep 2,4,8,16 400 600 | grep Threads || exit 1
timeout -k 10 120 bin/pe_cpu --backend omp --threads-sweep 4,8,16 800 1200 | grep Threads || exit 1
echo "## stage2 thread-ranks (reference process grid)"
for P in 2 4 8 16; do echo "P=$P: $(timeout -k 10 60 bin/pe_cpu --backend ranks --ranks $P --decomp reference 400 600 | grep Iter=)"; done
for P in 4 8 16; do echo "P=$P: $(timeout -k 10 120 bin/pe_cpu --backend ranks --ranks $P --decomp reference 800 1200 | grep Iter=)"; done
echo "## stage3 hybrid ranks x threads"
for c in "2 1" "2 2" "2 4" "2 8"; do set -- $c; echo "P=$1 T=$2: $(OMP_NUM_THREADS=$2 timeout -k 10 60 bin/pe_cpu --backend ranks --ranks $1 --threads $2 --decomp reference 400 600 | grep Iter=)"; done
for c in "4 1" "4 2" "4 4"; do set -- $c; echo "P=$1 T=$2: $(OMP_NUM_THREADS=$2 timeout -k 10 120 bin/pe_cpu --backend ranks --ranks $1 --threads $2 --decomp reference 800 1200 | grep Iter=)"; done
echo EXIT 0
