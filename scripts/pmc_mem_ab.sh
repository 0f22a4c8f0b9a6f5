#!/bin/bash
# Memory-side PMC A/B of library builds on the C2-shaped pass
# (scripts/probe_inflate.py): per build, L2 hit/miss and EA requests, wave
# wait/issue split and vector-memory instruction counts, per main dispatch of
# the inflate kernels (profiles/summarize.py).
# Usage (on the box, from the repo root): bash scripts/pmc_mem_ab.sh <tag> lib.so...
set -o pipefail
TAG=${1:-memab}; shift
N=${N:-10000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG/pmcmem
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  d=$OUT/v$i
  mkdir -p $d
  echo "$lib" > $d/lib.txt
  j=0
  for ctrs in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" \
              "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
    HBAM_LIB=$R/$lib HBAM_PROBE_CHILD=1 timeout -s KILL 240 rocprofv3 --pmc $ctrs \
      --output-format csv -d $d/p$j -o run -- python3 $R/scripts/probe_inflate.py $N > $d/probe$j.log 2> $d/err$j.log \
      || { echo "pmc pass $j failed for $lib"; tail -5 $d/err$j.log; exit 1; }
    j=$((j+1))
  done
  python3 - "$d" <<'PY'
import json, sys
sys.path.insert(0, sys.argv[1] + "/../../../../profiles")
import summarize
d = sys.argv[1]
lib = open(d + "/lib.txt").read().strip().split("/")[-1]
for k in ("hbam::k_inflate_huff", "hbam::k_inflate_lz77"):
    out = {"lib": lib, "kernel": k.split("::")[-1]}
    for p in ("p0", "p1"):
        c = summarize.counters(d, p, merge_instances=True).get(k, {})
        for n, v in c.items():
            if n.startswith("main:"):
                out[n[5:]] = round(v, 1) if v < 1e4 else int(v)
    print(json.dumps(out))
PY
  i=$((i+1))
done
