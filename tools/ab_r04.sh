#!/bin/bash
# one GPU call: the A/B rounds of tools/ab_lib.sh over the variants built locally
set -o pipefail
export VARIANTS="${VARIANTS:-base old}" ROUNDS="${ROUNDS:-3}" BENCH_ARGS="${BENCH_ARGS:---no-cpu-baseline}"
bash tools/ab_lib.sh
