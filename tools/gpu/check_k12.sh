set -u
# size-independent parity property on k = 12 mixed reads (configs[4]'s stress
# k): one device vs 4 virtual shards (multi-read pair-count blocks + owner
# reduce by lead) must give the identical dispatch
timeout -k 10 500 python bench.py --no-cpu-baseline --reads 1000000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --check-shards 4 > gpurun_out/chk_1m.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline --reads 2000000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --check-shards 4 > gpurun_out/chk_2m.log 2>&1 || exit 1
