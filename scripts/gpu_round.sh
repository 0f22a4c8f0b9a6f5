#!/bin/bash
# One GPU-box check of the tree: -m gpu tests, the C2 bench line (with the
# in-session PMC passes), and the N-rank launch rehearsed on one GPU.
# Usage (on the box, from the repo root): bash scripts/gpu_round.sh <tag> [steps...]
# steps: tests bench rehearsal (default: all three)
set -o pipefail
TAG=${1:-x}; shift
STEPS=${*:-tests bench rehearsal}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
      tail -2 $OUT/pytest_gpu.log ;;
    bench)
      timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 --no-extra > $OUT/bench.json 2> $OUT/bench.err \
        || { echo "bench failed"; tail -30 $OUT/bench.err; exit 2; }
      cat $OUT/bench.json ;;
    benchfull)
      timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err \
        || { echo "bench failed"; tail -30 $OUT/bench_full.err; exit 2; }
      cat $OUT/bench_full.json ;;
    reader)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_reader.py -x -q --timeout 120 --timeout-method thread \
        > $OUT/pytest_reader.log 2>&1 || { echo "reader tests failed"; tail -40 $OUT/pytest_reader.log; exit 1; }
      tail -2 $OUT/pytest_reader.log ;;
    hostlegs)
      timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-pmc --extras dropin_end_to_end --c3-gb 20 \
        > $OUT/bench_host.json 2> $OUT/bench_host.err || { echo "bench failed"; tail -30 $OUT/bench_host.err; exit 2; }
      python3 -c "import json,sys; d=json.load(open('$OUT/bench_host.json')); e=d['extra']; print(json.dumps(e['dropin_end_to_end'])); c=e['c3_c5_60GB']; print(json.dumps({k: c.get(k) for k in ('c3_streamed_from_host','value','matches_oracle')}))" ;;
    large)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_windows.py -x -q -s --timeout 500 \
        --timeout-method thread > $OUT/pytest_large.log 2>&1 || { echo "large tests failed"; tail -40 $OUT/pytest_large.log; exit 1; }
      tail -3 $OUT/pytest_large.log ;;
    qtrace)
      # which hardware queue each drop-in kernel and copy lands on, before and
      # after hbam_gpu_run_streamed (the slowed next context)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace \
        --output-format csv -d $OUT/qtrace -- python3 $R/scripts/dropin_probe2.py 10000000 --torch \
        --steps none,run_streamed,none,none > $OUT/qtrace.log 2>&1) \
        || { echo "qtrace failed"; tail -30 $OUT/qtrace.log; exit 4; }
      grep -E "^(mapped|resident)" $OUT/qtrace.log | cut -c1-300
      python3 scripts/qtrace_summary.py $OUT > $OUT/qtrace_summary.json 2>&1 || true
      python3 -c "import json; d=json.load(open('$OUT/qtrace_summary.json')); [print(k, json.dumps(v.get('overlap'))) for k, v in d.items() if isinstance(v, dict) and 'overlap' in v]" || true ;;
    dropin_ab)
      # the drop-in 1 M-batch loop under window ramps (HBAM_DROPIN_RAMP="first MiB,growth"; 0 = none)
      for r in ${RAMPS:-0 32,2}; do
        HBAM_DROPIN_RAMP=$r timeout -k 10 300 python -u scripts/dropin_probe2.py 10000000 --torch --steps none,none \
          > $OUT/dropin_ramp_$r.log 2>&1 || { echo "dropin probe failed"; tail -30 $OUT/dropin_ramp_$r.log; exit 6; }
        echo "ramp=$r"; grep -E "^(mapped|resident)" $OUT/dropin_ramp_$r.log | cut -c1-140
      done ;;
    feeds)
      # the drop-in 1 M-batch loop with fewer host copy threads staging the next window beside the batch D2H
      for f in ${FEEDS:-2 4 8}; do
        HBAM_FEED_THREADS=$f timeout -k 10 300 python -u scripts/dropin_probe2.py 10000000 --torch --steps none,none \
          > $OUT/dropin_feed_$f.log 2>&1 || { echo "dropin probe failed"; tail -30 $OUT/dropin_feed_$f.log; exit 6; }
        echo "feed threads=$f"; grep -E "^(mapped|resident)" $OUT/dropin_feed_$f.log | cut -c1-140
      done ;;
    envs)
      # the drop-in 1 M-batch loop under each VAR=VALUE of ENVS (runtime knobs)
      for e in ${ENVS:-NONE=0}; do
        env $e timeout -k 10 300 python -u scripts/dropin_probe2.py 10000000 --torch --steps none,none \
          > $OUT/dropin_env_$e.log 2>&1 || { echo "dropin probe failed"; tail -30 $OUT/dropin_env_$e.log; exit 6; }
        echo "env $e"; grep -E "^(mapped|resident)" $OUT/dropin_env_$e.log | cut -c1-140
      done ;;
    orderenvs)
      # the drop-in loop before and after hbam_gpu_run_streamed under each VAR=VALUE of ENVS
      for e in ${ENVS:-NONE=0}; do
        env $e timeout -k 10 300 python -u scripts/dropin_probe2.py 10000000 --torch --steps none,run_streamed,none,none \
          > $OUT/orderenv_$e.log 2>&1 || { echo "order probe failed"; tail -30 $OUT/orderenv_$e.log; exit 9; }
        echo "env $e"; grep -E "^(mapped|resident)" $OUT/orderenv_$e.log | cut -c1-110
      done ;;
    concurrent)
      # K FileVirtualSplits of C2 decoded at once by K contexts of one process (K map tasks per GPU)
      timeout -k 10 300 python -u scripts/concurrent_probe.py 10000000 ${KS:-1,2,3,4} > $OUT/concurrent.log 2>&1 \
        || { echo "concurrent probe failed"; tail -30 $OUT/concurrent.log; exit 13; }
      timeout -k 10 300 python -u scripts/concurrent_probe.py 10000000 ${KS:-1,2,3,4} --procs > $OUT/concurrent_procs.log 2>&1 \
        || { echo "concurrent probe (processes) failed"; tail -30 $OUT/concurrent_procs.log; exit 13; }
      cat $OUT/concurrent.log $OUT/concurrent_procs.log ;;
    fetchcalib)
      # FETCH_SIZE against the line bytes of known sparse access shapes (scripts/fetch_calib.hip)
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fcal \
        -o run -- $R/scripts/bin/fetch_calib > $OUT/fcal.log 2>&1) || { echo "fetch calib failed"; tail -20 $OUT/fcal.log; exit 14; }
      python3 scripts/fetch_calib_summary.py $OUT/fcal $OUT/fcal.log | tee $OUT/fcal_summary.txt ;;
    order)
      # the drop-in loop before and after hbam_gpu_run_streamed (the pinned-host leg), clocks and link sampled
      timeout -k 10 400 python -u scripts/dropin_probe2.py 10000000 --torch --smi --steps none,run_streamed,none,none \
        > $OUT/order.log 2>&1 || { echo "order probe failed"; tail -30 $OUT/order.log; exit 9; }
      grep -E "^(mapped|resident|SMI)" $OUT/order.log | cut -c1-260 ;;
    ordernuma)
      # the order probe with the NUMA placement of the process's large mappings before and after each loop
      timeout -k 10 400 python -u scripts/dropin_probe2.py 10000000 --numa --steps none,run_streamed,none,none \
        > $OUT/ordernuma.log 2>&1 || { echo "order probe failed"; tail -30 $OUT/ordernuma.log; exit 9; }
      grep -E "^(mapped|resident|NUMA)" $OUT/ordernuma.log | cut -c1-600 ;;
    orderrates)
      # torch's pinned copy rates beside the order probe's loops: is the slow state device-wide?
      timeout -k 10 400 python -u scripts/dropin_probe2.py 10000000 --torch --steps rates,run_streamed+rates,rates,rates \
        > $OUT/orderrates.log 2>&1 || { echo "order probe failed"; tail -30 $OUT/orderrates.log; exit 9; }
      grep -E "^(mapped|resident|RATES|prefetch)" $OUT/orderrates.log | cut -c1-300 ;;
    ordersteps)
      # which prior action triggers the slow mapped loop (STEPS: dropin_probe2 --steps list)
      timeout -k 10 500 python -u scripts/dropin_probe2.py 10000000 --torch --steps ${STEPS_LIST:-none,pinned_buffer,none,reload_pinned,none,none} \
        > $OUT/ordersteps.log 2>&1 || { echo "order probe failed"; tail -30 $OUT/ordersteps.log; exit 9; }
      grep -E "^(after|mapped|resident|prefetch)" $OUT/ordersteps.log | cut -c1-160 ;;
    ordertrace)
      # the same with the host-side timeline (HBAM_CURSOR_TRACE) of each loop
      HBAM_CURSOR_TRACE=1 timeout -k 10 400 python -u scripts/dropin_probe2.py 10000000 --torch \
        --steps none,run_streamed,none > $OUT/ordertrace.log 2> $OUT/ordertrace.err \
        || { echo "order trace failed"; tail -30 $OUT/ordertrace.err; exit 9; }
      grep -E "^(mapped|resident)" $OUT/ordertrace.log | cut -c1-200 ;;
    variants)
      # stage times + overlapped wall time per pass: the default build, the
      # in-tree experiment builds (lib/variants)
      timeout -k 10 400 python -u scripts/probe_inflate.py 10000000 hadoop-bam_amd/lib/libhbam.so \
        $(ls hadoop-bam_amd/lib/variants/*.so 2>/dev/null) > $OUT/variants.log 2>&1 \
        || { echo "variants failed"; tail -30 $OUT/variants.log; exit 5; }
      cat $OUT/variants.log ;;
    engines)
      # HIP log at level 4 (all categories; the copy lines name their engine): which DMA engine each copy of the drop-in loop
      # took, before and after hbam_gpu_run_streamed (the slowed next context)
      # (without torch: libhbam then loads /opt/rocm's HIP runtime, whose copy log names the engine)
      AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x7fffffff timeout -k 10 400 python -u scripts/dropin_probe2.py 10000000 \
        --steps none,run_streamed,none > $OUT/engines.log 2>&1 || { echo "engines probe failed"; tail -20 $OUT/engines.log; exit 12; }
      python3 scripts/engine_summary.py $OUT/engines.log > $OUT/engines.txt 2>&1
      grep -i "copy" $OUT/engines.log | head -c 2000000 > $OUT/engines_copylines.txt || true
      gzip -f $OUT/engines.log
      cat $OUT/engines.txt ;;
    gaps)
      # kernel trace of production-order passes (no events): overlap and idle time of the last pass
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gaps -o run \
        -- python3 $R/scripts/probe_inflate.py 10000000 > $OUT/gaps_probe.log 2>&1) || { echo "gaps trace failed"; tail -20 $OUT/gaps_probe.log; exit 11; }
      python3 scripts/pass_gaps.py $OUT/gaps > $OUT/gaps.txt 2>&1 || { echo "gaps analysis failed"; cat $OUT/gaps.txt; exit 11; }
      cat $OUT/gaps.txt ;;
    pmcab)
      # SQ issue / LDS counters of the inflate kernels per build (default + lib/variants)
      timeout -k 10 900 bash scripts/pmc_ab.sh $TAG > $OUT/pmcab.log 2>&1 || { echo "pmc a/b failed"; tail -20 $OUT/pmcab.log; exit 10; }
      cat $OUT/pmcab.log ;;
    dtrace)
      # host-side timeline of the drop-in 1 M-batch loop (window copies, decode
      # steps, batch issues, serial-link fallbacks)
      HBAM_CURSOR_TRACE=1 timeout -k 10 300 python -u scripts/dropin_probe2.py 10000000 --torch --steps none,none \
        > $OUT/dtrace.log 2> $OUT/dtrace.err || { echo "dtrace failed"; tail -30 $OUT/dtrace.err; exit 7; }
      grep -E "^(mapped|resident)" $OUT/dtrace.log | cut -c1-160; (grep -c "serial link" $OUT/dtrace.err || true)
      HBAM_CURSOR_TRACE=1 timeout -k 10 200 python -u scripts/probe_inflate.py 10000000 > $OUT/ptrace.log \
        2> $OUT/ptrace.err || { echo "ptrace failed"; tail -30 $OUT/ptrace.err; exit 7; }
      (grep -A3 "chain\]" $OUT/dtrace.err | head -40; grep "chain\]" $OUT/ptrace.err | head -24) || true ;;
    collect)
      # rocprofv3 kernel trace + stats and the PMC passes of bench.py --serial (profiles/collect.sh)
      timeout -k 10 900 bash profiles/collect.sh $TAG > $OUT/collect.log 2>&1 \
        || { echo "collect failed"; tail -30 $OUT/collect.log; exit 8; }
      python3 -c "import json; d=json.load(open('$R/gpurun_out/prof_$TAG/summary.json'))['kernels']; [print('%-45s calls %4d main_avg_us %9.1f' % (k[:45], v['calls'], v.get('main_avg_ns', 0) / 1e3)) for k, v in sorted(d.items(), key=lambda x: -x[1].get('total_ns', 0))[:22]]" ;;
    rehearsal)
      timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --one-device --c3-gb 7 --steps 3 --warmup 1 \
        > $OUT/rehearsal.json 2> $OUT/rehearsal.err || { echo "rehearsal failed"; tail -30 $OUT/rehearsal.err; exit 3; }
      cat $OUT/rehearsal.json ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 15; }
      tail -2 $OUT/smoke.log ;;
    rehearsal8)
      # the driver's 8-GPU sequence with 8 gloo ranks sharing this box's one GPU
      timeout -k 10 900 python -u bench.py --gpus 8 --dist-backend gloo --one-device --c3-gb 4 --steps 3 --warmup 1 \
        > $OUT/rehearsal8.json 2> $OUT/rehearsal8.err || { echo "rehearsal8 failed"; tail -30 $OUT/rehearsal8.err; exit 3; }
      cat $OUT/rehearsal8.json ;;
  esac
done
