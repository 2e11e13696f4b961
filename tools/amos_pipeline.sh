#!/bin/bash
# AMOS pipeline acceptance harness: the reference's
# `rake project` pipe (Rakefile.rb:164-215) with sa-overlap as the overlapper,
# in two forms:
#   ovl  toAmos_new -s X.seq -b X.bnk ; sa-overlap -i X.seq -o X.ovl ;
#        bank-transact -b X.bnk -m X.ovl                       (the Rakefile's order)
#   afg  sa-overlap -i X.seq -o X.ovl --afg X.afg ; bank-transact -c -b X.bnk -m X.afg
#        (the bank's reads and overlaps from one message file: no toAmos_new)
# then tigger -b X.bnk ; make-consensus -e 0.04 -o 40 -B -b X.bnk ;
# bank2fasta -b X.bnk > X.fasta, and the contig is compared with EXPECTED.
#
# Usage: tools/amos_pipeline.sh AMOS_BIN_DIR X.seq EXPECTED.fasta [ovl|afg] [sa-overlap flags...]
# AMOS_BIN_DIR must hold AMOS builds the user supplies: the prebuilt binaries
# inside the reference are never run by this repository (so neither the tests
# nor the GPU sessions call this script).
set -euo pipefail
AMOS=$1; SEQ=$2; EXPECTED=$3; FORM=${4:-afg}; shift 3; if [ $# -gt 0 ]; then shift; fi
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SA=$ROOT/sequence-aligner_amd/build/sa-overlap
WORK=$(mktemp -d)
trap 'rm -rf "$WORK"' EXIT
raw=$(basename "${SEQ%.*}")
cp "$SEQ" "$WORK/$raw.seq"
cd "$WORK"
t0=$(date +%s.%N)
if [ "$FORM" = ovl ]; then
    "$AMOS/toAmos_new" -s "$raw.seq" -b "$raw.bnk"
    "$SA" -i "$raw.seq" -o "$raw.ovl" "$@"
    "$AMOS/bank-transact" -b "$raw.bnk" -m "$raw.ovl"
else
    "$SA" -i "$raw.seq" -o "$raw.ovl" --afg "$raw.afg" "$@"
    "$AMOS/bank-transact" -c -b "$raw.bnk" -m "$raw.afg"
fi
t1=$(date +%s.%N)
"$AMOS/tigger" -b "$raw.bnk"
"$AMOS/make-consensus" -e 0.04 -o 40 -B -b "$raw.bnk"
"$AMOS/bank2fasta" -b "$raw.bnk" > "$raw.fasta"
t2=$(date +%s.%N)
echo "overlap + bank: $(echo "$t1 - $t0" | bc) s, layout + consensus + fasta: $(echo "$t2 - $t1" | bc) s"
if cmp -s "$raw.fasta" "$EXPECTED"; then
    echo "contig identical to $EXPECTED"
else
    echo "contig differs from $EXPECTED" >&2
    exit 1
fi
