set -u
# configs[3] / configs[4] k=15 per-GPU slices on the tree with the wave pair counter
bash tools_slice_prof.sh c3 --reads 1250000 --steps 3 --warmup 1 --align-steps 1 || exit 1
bash tools_slice_prof.sh c4k15 --reads 6250000 --len 1000 --min-len 100 --k 15 --steps 2 --warmup 1 --align-steps 1 || exit 1
