#!/bin/bash
# Same-box A/B over variant library builds (a fresh process each, alternating):
#   VARIANTS="dir[:ENV=v[,ENV=v]] ..."  directories under sequence-aligner_amd/ holding
#                      a libsa_overlap.so (make OUT=build_x EXTRA=-D...), each with
#                      optional environment knobs, e.g. "build build:SA_MAIN_CAP=2048"
#   REPS=3 rounds;  ARGS="..." extra bench.py arguments;  AB_TIMEOUT=120 per run
# One line per run into gpurun_out/ab.txt: variant, hash step, sort, buckets,
# pairs, align step, align kernel, emit (ms).  Run from the repository root.
set -u
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
 for v in $VARIANTS; do
  dir=${v%%:*}
  envs=""
  [ "$dir" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
  env SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$dir/libsa_overlap.so $envs timeout -k 10 ${AB_TIMEOUT:-120} python bench.py --steps 8 --warmup 2 --no-cpu-baseline --align-steps 6 ${ARGS:-} > gpurun_out/ab_run.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/ab_run.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], s["sort"], s["buckets"], s["pairs"], d["ms_per_align_step"], d["align_kernel_ms"], s["emit"])')" >> gpurun_out/ab.txt
 done
done
