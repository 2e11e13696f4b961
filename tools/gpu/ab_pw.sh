#!/bin/bash
# wave pair-counter shape A/B: chunk 128 / batch 8 (tree) vs chunk 64, 256 and batch 16
VARIANTS="build build_pw64 build_pw256 build_pwb16 build_pw64b16" REPS=3 timeout -k 10 600 bash tools/gpu/ab_multi.sh
