set -euo pipefail
export TMPDIR=/tmp
bash tools/prof.sh r02b
timeout -k 10 600 python3 bench.py > gpurun_out/prof_r02b/bench_default.json 2>gpurun_out/prof_r02b/bench_default.err
tail -1 gpurun_out/prof_r02b/bench_default.json
