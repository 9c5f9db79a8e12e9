set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc_run.log 2>&1 || { tail -30 gpurun_out/pmc_run.log; exit 1; }
tail -3 gpurun_out/pmc_run.log | cut -c1-300
