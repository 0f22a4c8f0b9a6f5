#!/bin/bash
# PMC A/B of library builds on the C2-shaped pass (scripts/probe_inflate.py):
# one rocprofv3 --pmc run per build with the SQ issue / LDS counters, then the
# per-kernel averages of the main dispatches (profiles/summarize.py).
# Usage (on the box, from the repo root): bash scripts/pmc_ab.sh <tag> [records]
set -o pipefail
TAG=${1:-ab}
N=${2:-10000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for lib in $R/hadoop-bam_amd/lib/libhbam.so $(ls $R/hadoop-bam_amd/lib/variants/*.so 2>/dev/null); do
  d=$OUT/v$i
  mkdir -p $d
  echo "$lib" > $d/lib.txt
  HBAM_LIB=$lib HBAM_PROBE_CHILD=1 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d $d/sq -o run -- python3 $R/scripts/probe_inflate.py $N > $d/probe.log 2> $d/err.log \
    || { echo "pmc pass failed for $lib"; tail -5 $d/err.log; exit 1; }
  python3 - "$d" <<'EOF'
import json, sys
sys.path.insert(0, sys.argv[1] + "/../../../../profiles")
import summarize
d = sys.argv[1]
cs = summarize.counters(d, "sq", merge_instances=True)
lib = open(d + "/lib.txt").read().strip().split("/")[-1]
for k in ("hbam::k_inflate_huff", "hbam::k_inflate_lz77", "hbam::k_huff_tables"):
    c = cs.get(k, {})
    g = lambda n: c.get("main:" + n, 0.0)
    cyc = g("GRBM_GUI_ACTIVE") / 8 or 1
    out = {"lib": lib, "kernel": k.split("::")[-1], "dispatches": c.get("main_dispatches"),
           "valu": int(g("SQ_INSTS_VALU")), "salu": int(g("SQ_INSTS_SALU")), "lds": int(g("SQ_INSTS_LDS")),
           "valu_frac": round(g("SQ_INSTS_VALU") * 2 / (1024 * cyc), 3),
           "lds_frac": round(g("SQ_LDS_IDX_ACTIVE") / (256 * cyc), 3),
           "conf_per_lds": round(g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_INSTS_LDS"), 1), 3),
           "ldscyc_per_lds": round(g("SQ_LDS_IDX_ACTIVE") / max(g("SQ_INSTS_LDS"), 1), 3),
           "wait_lds_frac": round(g("SQ_WAIT_INST_LDS") / max(g("SQ_WAVE_CYCLES"), 1), 3),
           "valu_active_frac": round(g("SQ_ACTIVE_INST_VALU") / max(g("SQ_WAVE_CYCLES"), 1), 3),
           "cycles": int(cyc)}
    print(json.dumps(out))
EOF
  i=$((i+1))
done
