set -euo pipefail
out=gpurun_out/r02z
mkdir -p $out
export TMPDIR=/tmp LZ4MT_BENCH_BACKEND=gloo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --gib 1 --steps 2 --warmup 1 > $out/n2.json 2> $out/n2.err
tail -1 $out/n2.json
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 3 --gib 0.5 --steps 2 --warmup 1 > $out/n3.json 2> $out/n3.err
tail -1 $out/n3.json
