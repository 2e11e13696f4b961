set -u
# configs[3] / configs[4] per-GPU slices on the current tree, each with kernel
# stats and PMC passes keyed to its workload (tools_slice_prof.sh)
bash tools_slice_prof.sh c3 --reads 1250000 --steps 3 --warmup 1 --align-steps 1 || exit 1
bash tools_slice_prof.sh c4k15 --reads 6250000 --len 1000 --min-len 100 --k 15 --steps 2 --warmup 1 --align-steps 1 || exit 1
bash tools_slice_prof.sh c4k12 --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 || exit 1
