#!/bin/bash
# One GPU-box pass for a round: any of the steps below, in the order given,
# each under its own time limit; the first failure ends the pass.
# usage (from the repo root on the box): bash tools/gpu_round.sh <tag> <step>...
#   tests   pytest -m gpu (every GPU test file)
#   tdist   pytest -m gpu tests/test_gpu_dist.py (the multi-rank paths) only
#   bench   the default 1-GPU bench line (driver shape: --steps 20 --warmup 5)
#   trace   rocprofv3 kernel-trace stats of a 5-step bench run
#   sq      SQ counters of the encoder / decoder (tools/kprof.py 2) + the window count (tools/kstats.py 2)
#   pmc     FETCH_SIZE / WRITE_SIZE passes (tools/prof.sh without its trace)
#   pmc32   the same at 32 GiB (configs[2]'s decompress traffic, tools/pmcsum.py --gib=32)
#   pmcbid  the same on App. F at block ids 4, 5, 6 (the configs[4] sweep: profiles/pmc_b<id>.json)
#   dist2   bench.py --gpus 2 over gloo on this one GPU (rehearsal of the N > 1 path)
#   fcal    FETCH_SIZE calibration on a known byte count (tools/fetch_cal.py + fetchcal_sum.py)
#   unpack  the root's unpack from each IPC receive-buffer memory kind (tools/unpack_ab.py)
#   tail    the streamed gather's exposed tail on one GPU (tools/tail_model.py)
#   ab      kernel times of every exp_libs/*.so (tools/mkvariants.sh), two passes
#   abtrace kernel-trace stats of every exp_libs/*.so;  abbid  ab at every block size
#   fuzz    random differential campaign (300 s);  sweep  the secondary bench configs
#   probe   k_encode with the exchange probe vs the read-back fallback
#   e2ems   end-to-end memory path: streamed compress vs the batch engine
#   e2e     end-to-end rates (tools/e2e.py 8 7: host memory, then file -> file in /dev/shm)
#   occ     encoder time against resident waves per CU (tools/occ_sweep.py)
#   ovl     the split parse's parse work with real overlap (occ_sweep.py --overlap)
#   bdref   the -BD reference-bytes tests (tests/test_gpu_bd.py -k reference)
#   tstream the streamed callback compress tests + the callback-engine config tests
#   nccl1   the world-size-1 nccl tests (tests/test_gpu_dist.py -k nccl)
#   interf  k_encode at 8 vs 4 waves per CU (LDS pad) at B7 / B6: what two waves per SIMD cost each other
set -euo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 1100 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests \
          > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
      tail -2 "$out/pytest.log" ;;
    tdist)
      timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py \
          > "$out/pytest_dist.log" 2>&1 || { tail -40 "$out/pytest_dist.log"; exit 1; }
      tail -2 "$out/pytest_dist.log" ;;
    bench)
      timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
      cat "$out/bench.json" ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$out/trace" -o trace -- \
          python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > "$out/trace_bench.json" 2> "$out/trace.err"
      cat "$out/trace_bench.json" ;;
    sq)
      timeout -k 10 200 python3 tools/kstats.py 2 > "$out/kstats.txt" 2>&1
      head -3 "$out/kstats.txt"
      timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM \
          SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -T -f csv -d "$out/sq" -o sq -- \
          python3 tools/kprof.py 2 > "$out/sq.log" 2>&1
      python3 tools/sqsum.py "$out/sq" "$out/kstats.txt" | tee "$out/sq_summary.txt" ;;
    pmc)
      for input in appf random; do
        flag=""; [ "$input" = random ] && flag="--random"
        timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -f csv -d "$out/fetch_$input" -o fetch -- \
            python3 tools/kprof.py 8 $flag > "$out/fetch_$input.log" 2>&1
        timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -T -f csv -d "$out/write_$input" -o write -- \
            python3 tools/kprof.py 8 $flag > "$out/write_$input.log" 2>&1
      done ;;
    pmcbid)
      for bid in 4 5 6; do
        mkdir -p "$out/bid$bid"
        timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -f csv -d "$out/bid$bid/fetch_appf" -o fetch -- \
            python3 tools/kprof.py 8 --bid=$bid > "$out/bid$bid/fetch.log" 2>&1
        timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -T -f csv -d "$out/bid$bid/write_appf" -o write -- \
            python3 tools/kprof.py 8 --bid=$bid > "$out/bid$bid/write.log" 2>&1
      done ;;
    e2ems)   # end-to-end memory path, the streamed engines (default) and the batch engine (LZ4MT_AMD_STREAM=0)
      timeout -k 10 300 python3 tools/e2e.py 8 7 > "$out/e2e_mem_stream.txt" 2>&1 || { tail -20 "$out/e2e_mem_stream.txt"; exit 1; }
      LZ4MT_AMD_STREAM=0 timeout -k 10 300 python3 tools/e2e.py 8 7 > "$out/e2e_mem_batch.txt" 2>&1 \
          || { tail -20 "$out/e2e_mem_batch.txt"; exit 1; }
      grep e2e "$out/e2e_mem_stream.txt" | sed 's/^/streamed: /'; grep e2e "$out/e2e_mem_batch.txt" | sed 's/^/batch: /' ;;
    pmc32)   # FETCH_SIZE / WRITE_SIZE of a 32 GiB App. F compress + decompress (configs[2]'s decode traffic)
      mkdir -p "$out/p32"
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -f csv -d "$out/p32/fetch_appf" -o fetch -- \
          python3 tools/kprof.py 32 > "$out/fetch_32.log" 2>&1
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -T -f csv -d "$out/p32/write_appf" -o write -- \
          python3 tools/kprof.py 32 > "$out/write_32.log" 2>&1
      tail -1 "$out/fetch_32.log" ;;
    e2e)
      timeout -k 10 300 python3 tools/e2e.py 8 7 > "$out/e2e_mem.txt" 2>&1 || { tail -20 "$out/e2e_mem.txt"; exit 1; }
      cat "$out/e2e_mem.txt"
      mkdir -p /dev/shm/lz4mt_e2e
      timeout -k 10 400 python3 tools/e2e.py 8 7 --file /dev/shm/lz4mt_e2e > "$out/e2e_file.txt" 2>&1 \
          || { rm -rf /dev/shm/lz4mt_e2e; tail -20 "$out/e2e_file.txt"; exit 1; }
      rm -rf /dev/shm/lz4mt_e2e
      cat "$out/e2e_file.txt" ;;
    ovl)
      timeout -k 10 400 python3 tools/occ_sweep.py --overlap > "$out/ovl.txt" 2>&1 || { tail -20 "$out/ovl.txt"; exit 1; }
      cat "$out/ovl.txt" ;;
    occ)
      timeout -k 10 400 python3 tools/occ_sweep.py > "$out/occ.txt" 2>&1 || { tail -20 "$out/occ.txt"; exit 1; }
      cat "$out/occ.txt" ;;
    bdref)
      timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_bd.py \
          -k reference > "$out/pytest_bdref.log" 2>&1 || { tail -40 "$out/pytest_bdref.log"; exit 1; }
      tail -3 "$out/pytest_bdref.log" ;;
    tstream)   # the streamed callback compress (tests/test_gpu_stream.py) and the callback-engine tests
      timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py \
          tests/test_gpu_configs.py > "$out/pytest_stream.log" 2>&1 || { tail -40 "$out/pytest_stream.log"; exit 1; }
      tail -3 "$out/pytest_stream.log" ;;
    nccl1)
      timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py \
          -k nccl > "$out/pytest_nccl1.log" 2>&1 || { tail -40 "$out/pytest_nccl1.log"; exit 1; }
      tail -3 "$out/pytest_nccl1.log" ;;
    dist2)
      LZ4MT_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --gib 0.5 --steps 2 --warmup 1 \
          --no-cpu-baseline > "$out/dist2.json" 2> "$out/dist2.err"
      cat "$out/dist2.json" ;;
    fcal)
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -f csv -d "$out/fcal" -o fcal -- \
          python3 tools/fetch_cal.py 8 > "$out/fcal.log" 2>&1
      python3 tools/fetchcal_sum.py "$out/fcal" 8 | tee "$out/fcal_summary.json" ;;
    unpack)   # the root's unpack cost per receive-buffer memory kind (tools/unpack_ab.py)
      timeout -k 10 200 python3 tools/unpack_ab.py 8 > "$out/unpack_ab.json" 2> "$out/unpack_ab.err" \
          || { tail -20 "$out/unpack_ab.err"; exit 1; }
      cat "$out/unpack_ab.json" ;;
    tail)
      timeout -k 10 300 python3 tools/tail_model.py 8 8 > "$out/tail_model.txt" 2>&1
      cat "$out/tail_model.txt" ;;
    tailab)   # tools/tail_model.py for every exp_libs/*.so
      for f in exp_libs/*.so; do
        echo "== $f" >> "$out/tail_ab.txt"
        LZ4MT_AMD_LIB=$f timeout -k 10 300 python3 tools/tail_model.py 8 8 2>&1 | grep -v amdgpu >> "$out/tail_ab.txt"
      done
      cat "$out/tail_ab.txt" ;;
    ab)
      bash tools/ab.sh > "$out/ab.txt" 2>&1 && bash tools/ab.sh >> "$out/ab.txt" 2>&1
      cat "$out/ab.txt" ;;
    follow)   # block checksums beside the encode (LZ4MT_AMD_FOLLOW=1) vs after it (the default), twice each
      for k in 1 2; do
        for f in 1 0; do
          LZ4MT_AMD_FOLLOW=$f timeout -k 10 120 python3 -u tools/ktime.py 2>&1 | grep -v amdgpu | sed "s/^/FOLLOW=$f /" \
              >> "$out/follow.txt"
        done
      done
      cat "$out/follow.txt" ;;
    abpar)   # quick parity screen (tools/abparity.py) of every exp_libs/*.so; mismatches are reported, not fatal
      for f in exp_libs/*.so; do
        LZ4MT_AMD_LIB_OLDER=1 LZ4MT_AMD_LIB=$f timeout -k 10 200 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu \
            >> "$out/abpar.txt" || true
      done
      cat "$out/abpar.txt" ;;
    abtest)   # parity tests against exp_libs/$ABLIB.so (the candidate of an A/B)
      LZ4MT_AMD_LIB=exp_libs/$ABLIB.so timeout -k 10 900 python3 -u -m pytest -m gpu -x -q --timeout 300 \
          --timeout-method thread tests/test_gpu.py tests/test_gpu_configs.py tests/test_gpu_bd.py \
          > "$out/abtest_$ABLIB.log" 2>&1 || { tail -30 "$out/abtest_$ABLIB.log"; exit 1; }
      tail -2 "$out/abtest_$ABLIB.log" ;;
    ab5)   # the same at 256 KiB blocks (32768 blocks per 8 GiB: occupancy-sensitive)
      BID=5 bash tools/ab.sh > "$out/ab5.txt" 2>&1 && BID=5 bash tools/ab.sh >> "$out/ab5.txt" 2>&1
      cat "$out/ab5.txt" ;;
    abtrace)   # kernel-trace stats of tools/ktime.py for every exp_libs/*.so (per-kernel times per variant)
      for f in exp_libs/*.so; do
        nm=$(basename $f .so)
        LZ4MT_AMD_LIB=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d "$out/$nm" -o t -- \
            python3 tools/ktime.py > "$out/$nm.txt" 2>&1
        grep -v amdgpu "$out/$nm.txt"
      done ;;
    abbid)   # tools/ab.sh at BID = 4, 6, 5, 7 (block-size dependence of an A/B)
      for b in 4 6 5 7; do
        echo "## BID $b" >> "$out/ab_bid.txt"
        BID=$b bash tools/ab.sh >> "$out/ab_bid.txt" 2>&1
      done
      cat "$out/ab_bid.txt" ;;
    probe)   # kernel times with the exchange probe (default) and the read-back fallback (LZ4MT_AMD_ENC_PROBE=readback)
      for i in 1 2; do
        timeout -k 10 200 python3 tools/ktime.py 2>&1 | tail -1 | sed 's/^/exchange  /' | tee -a "$out/probe.txt"
        LZ4MT_AMD_ENC_PROBE=readback timeout -k 10 200 python3 tools/ktime.py 2>&1 | tail -1 | sed 's/^/read-back /' \
            | tee -a "$out/probe.txt"
      done ;;
    fuzz)   # time-boxed random differential campaign (seed 7) against the oracle / liblz4
      timeout -k 10 420 python3 -u tools/fuzz_campaign.py 300 ${FUZZ_SEED:-7} > "$out/fuzz.txt" 2>&1
      tail -2 "$out/fuzz.txt" ;;
    sweep)   # secondary configs: block sizes, 32 GiB decompress-only, default flags, HC level 9, -BD B7
      for spec in "b4 --block-id 4 --steps 5 --warmup 2" "b5 --block-id 5 --steps 5 --warmup 2" \
                  "b6 --block-id 6 --steps 5 --warmup 2" "dec32 --gib 32 --decompress-only --steps 3 --warmup 1" \
                  "sck --stream-checksum --steps 3 --warmup 1" "hc9 --level 9 --steps 2 --warmup 1" \
                  "bd7 --block-dependent --steps 2 --warmup 1"; do
        set -- $spec; name=$1; shift
        timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$out/$name.json" 2> "$out/$name.err"
        echo "$name $(cut -c1-300 "$out/$name.json")"
      done ;;
    interf)  # the encoder's waves interfering on a SIMD: 8 waves per CU (2 per SIMD) vs 4 (LDS padded, 1 per SIMD)
      for bid in 7 6; do
        for pad in 0 20480; do
          LZ4MT_AMD_ENC_LDS_PAD=$pad BID=$bid KTIME_NOCHECK=0 timeout -k 10 200 python3 tools/ktime.py \
              > "$out/interf_b${bid}_pad$pad.txt" 2>&1 || { tail -5 "$out/interf_b${bid}_pad$pad.txt"; exit 1; }
          echo "B$bid pad $pad: $(grep encode "$out/interf_b${bid}_pad$pad.txt")"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
