# encoder scheduler A/B per block size (tools/ab.sh with BID = 4, 5, 6, 7)
set -euo pipefail
mkdir -p gpurun_out/r03y
for b in 4 6 5 7; do
  echo "## BID $b" >> gpurun_out/r03y/ab.txt
  BID=$b bash tools/ab.sh >> gpurun_out/r03y/ab.txt 2>&1
done
cat gpurun_out/r03y/ab.txt
