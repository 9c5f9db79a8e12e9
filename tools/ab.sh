#!/bin/bash
# A/B timing on one GPU box: the bench line of this tree ("base") against
# full trees under ab/<name>/ (other revisions, e.g. `git worktree add ab/x`,
# each with its own built library). Rounds alternate, so drift hits every arm
# alike. The product sources carry no A/B switches: a variant is a revision.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 2000 --warmup 300 --no-cpu-baseline"}
for round in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ -d "ab/$v" ]; then
      (cd "ab/$v" && timeout -k 10 120 python bench.py $ARGS) > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.log || exit 1
    else
      timeout -k 10 120 python bench.py $ARGS > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.log || exit 1
    fi
    python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('r$round $v', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,3), 'us/step kernel', round(d['roofline']['kernel_avg_us'],3))"
  done
done
echo ab done
