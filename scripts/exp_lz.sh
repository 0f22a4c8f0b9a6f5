# Experiment: phase-B variants (lib/variants/*.so): cycle profile + bench.
# usage: bash scripts/exp_lz.sh default ilp1 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = default ]; then unset HBAM_LIB; else export HBAM_LIB=$PWD/hadoop-bam_amd/lib/variants/libhbam_$v.so; fi
  echo "== $v"
  HBAM_INFLATE_SERIAL=1 HBAM_HUFF_PROF=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 1 --warmup 0 > gpurun_out/l_$v.json 2> gpurun_out/l_$v.err || { tail gpurun_out/l_$v.err; exit 1; }
  grep "lz77 prof" gpurun_out/l_$v.err | tail -1
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 5 --warmup 1 > gpurun_out/lb_$v.json 2>gpurun_out/lb_$v.err || { tail gpurun_out/lb_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stages_ms'])" gpurun_out/lb_$v.json
done
