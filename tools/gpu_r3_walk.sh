#!/bin/bash
# Walk-variant study: parity subset + isolated-walk timing of each study build
# in emqx_amd/variants (tools/gpu_variants.sh), then kernel-trace passes for
# the builds named in LIBS (default: all).  usage: tools/gpu_r3_walk.sh <tag>
set -e
bash tools/gpu_variants.sh $1 --batches 16
