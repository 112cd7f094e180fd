# final-build profiles (bench, kernel trace, PMC), then the HC object scheduler A/B (tools/abhc.sh)
set -euo pipefail
bash tools/gpu_round.sh r03u bench trace pmc
timeout -k 10 900 bash tools/abhc.sh hcilp r03u_hc
cat gpurun_out/r03u_hc/ab.txt; tail -2 gpurun_out/r03u_hc/tests.log
