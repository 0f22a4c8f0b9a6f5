#!/bin/bash
# bench.py --no-extra (timed, overlapped order) once per library variant.
# usage: bash scripts/bench_variants.sh lib1.so lib2.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
for LIB in "$@"; do
  HBAM_LIB=$R/$LIB timeout -k 10 300 python3 $R/bench.py --no-extra --no-cpu-baseline --no-pmc 2>/dev/null | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$LIB', d['value'], d['ms_per_step'], d['stages_ms'])" || exit 1
done
