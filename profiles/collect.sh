#!/bin/bash
# Collect the rocprofv3 evidence for one round on the GPU box:
#   1. kernel trace + stats (per-kernel average durations)
#   2. PMC pass FETCH_SIZE, 3. PMC pass WRITE_SIZE (separate passes: TCC slots)
#   4. PMC pass of SQ counters (VALU / LDS / bank conflicts / occupancy)
# then summarises everything into $OUT/summary.json (profiles/summarize.py).
# Only the C2 headline runs under the profiler (--no-extra): the side
# measurements would add launches of other sizes to the per-kernel averages.
# --serial: every step in the measurement launch order (one stream), so the
# per-kernel averages are the kernel durations bench.py's roofline uses.
# Usage (from the repo root on the box): bash profiles/collect.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --no-cpu-baseline --no-extra --no-pmc --serial $*"
PMCB="python3 $R/bench.py --no-cpu-baseline --no-extra --no-pmc --serial --steps 1 --warmup 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH \
  > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace pass failed"; tail -5 $OUT/trace.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $PMCB \
  > /dev/null 2> $OUT/fetch.err || { echo "FETCH_SIZE pass failed"; tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $PMCB \
  > /dev/null 2> $OUT/write.err || { echo "WRITE_SIZE pass failed"; tail -5 $OUT/write.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- $PMCB \
  > /dev/null 2> $OUT/sq.err || { echo "SQ pass failed"; tail -5 $OUT/sq.err; exit 1; }
python3 $R/profiles/summarize.py $OUT > $OUT/summary.json && cat $OUT/summary.json
