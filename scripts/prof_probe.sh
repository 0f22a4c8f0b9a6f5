#!/bin/bash
# Kernel trace + SQ counters of scripts/probe_inflate.py (one lib) on the GPU box.
# usage: bash scripts/prof_probe.sh <tag> [records] [lib.so]
set -o pipefail
TAG=${1:-p}; N=${2:-10000000}; LIB=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/probe_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export HBAM_LIB=$R/$LIB
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/scripts/probe_inflate.py $N > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- \
  python3 $R/scripts/probe_inflate.py $N > $OUT/sq.log 2>&1 || { echo "SQ failed"; tail -5 $OUT/sq.log; exit 1; }
python3 $R/profiles/summarize.py $OUT > $OUT/summary.json && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k, {x: (round(y,3) if isinstance(y,float) else y) for x,y in v.items() if x in (\"calls\",\"avg_ns\",\"main_avg_ns\",\"total_ns\",\"valu_active_frac_of_wave_cycles\",\"lds_bank_conflict_per_lds_inst\",\"SQ_INSTS_VALU\",\"SQ_INSTS_LDS\",\"SQ_WAVES\")}) for k,v in list(d[\"kernels\"].items())[:12]]; print(d[\"inflate_stage\"])" $OUT/summary.json
