# Experiment: phase-A variants (lib/variants/*.so) with the per-block cycle profile.
# usage: bash scripts/exp_huff_variants.sh default m2 m8 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = default ]; then unset HBAM_LIB; else export HBAM_LIB=$PWD/hadoop-bam_amd/lib/variants/libhbam_$v.so; fi
  echo "== $v"
  HBAM_HUFF_PROF=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/b_$v.json 2> gpurun_out/b_$v.err || { tail gpurun_out/b_$v.err; exit 1; }
  grep "huff prof" gpurun_out/b_$v.err | tail -1
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['stages_ms'])"
done
