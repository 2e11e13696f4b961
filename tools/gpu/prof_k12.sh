set -u
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p_k12 -o run -- python3 $R/bench.py --no-cpu-baseline --reads 1000000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 > $R/gpurun_out/p_k12.log 2>&1 || exit 1
