set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -5
