# Bench (with the C4 side measurement) for each variant library: default or lib/variants/libhbam_<v>.so
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = default ]; then unset HBAM_LIB; else export HBAM_LIB=$PWD/hadoop-bam_amd/lib/variants/libhbam_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/v_$v.json 2> gpurun_out/v_$v.err || { tail gpurun_out/v_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stages_ms']); print('C4', d['extra']['c4_long_reads'])" gpurun_out/v_$v.json
done
