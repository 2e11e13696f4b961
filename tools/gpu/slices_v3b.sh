set -u
# configs[4] k=12 per-GPU slice (the LDS-occupancy stress) on the tree with the wave pair counter
bash tools_slice_prof.sh c4k12 --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 || exit 1
