# Experiment: overlapped phase A/B inflate variants vs HBAM_INFLATE_SERIAL=1.
# usage: bash scripts/exp_overlap.sh default ns6 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = default ]; then unset HBAM_LIB; else export HBAM_LIB=$PWD/hadoop-bam_amd/lib/variants/libhbam_$v.so; fi
  for ser in 0 1; do
    if [ $ser = 1 ]; then export HBAM_INFLATE_SERIAL=1; else unset HBAM_INFLATE_SERIAL; fi
    echo "== $v serial=$ser"
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 5 --warmup 1 > gpurun_out/o_$v$ser.json 2> gpurun_out/o_$v$ser.err || { tail gpurun_out/o_$v$ser.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stages_ms'])" gpurun_out/o_$v$ser.json
  done
done
