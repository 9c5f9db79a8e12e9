set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="base rankonly norefill" bash tools/ab.sh || exit 1
