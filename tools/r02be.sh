# full GPU suite + smoke after the HC optimal-parser work
set -euo pipefail
out=gpurun_out/r02be
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > $out/tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
