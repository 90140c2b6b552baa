#!/bin/bash
# Deep-topic hand-over without the scan of the rest (study build deepskip) vs
# the product copy: parity subset, then the isolated walk on C3deep and C3.
# usage: tools/gpu_deepskip.sh <tag>
set -e
bash tools/gpu_variants.sh $1 --config c3deep --batches 16
NOTEST=1 bash tools/gpu_variants.sh $1 --config c3 --batches 16
