#!/bin/bash
# Kernel trace of scripts/probe_inflate.py once per library variant.
# usage: bash scripts/trace_variants.sh <tag> <records> lib1.so lib2.so ...
set -o pipefail
TAG=$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for LIB in "$@"; do
  V=$(basename $LIB .so)
  OUT=$R/gpurun_out/tv_$TAG/$V
  mkdir -p $OUT
  HBAM_LIB=$R/$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/scripts/probe_inflate.py $N > $OUT/trace.log 2>&1 || { echo "$V failed"; tail -5 $OUT/trace.log; exit 1; }
  python3 $R/profiles/summarize.py $OUT > $OUT/summary.json || exit 1
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))['kernels']
print(sys.argv[2], {k.replace('hbam::',''): round(v['total_ns']/6e6,3) for k,v in d.items() if 'inflate' in k or 'huff' in k})" $OUT/summary.json $V
done
