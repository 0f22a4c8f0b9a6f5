# Per-block cycle profiles (phase A + phase B) need a library built with the
# accumulators compiled in:
#   make -C hadoop-bam_amd BUILD=build_kprof LIBOUT=lib/variants/libhbam_kprof.so EXTRA=-DHBAM_KPROF=1
# then: bash scripts/exp_lzprof.sh kprof
# Timing-only phase-B experiments (variants may produce wrong bytes): prints the cycle profile.
for v in "$@"; do
  if [ $v = default ]; then unset HBAM_LIB; else export HBAM_LIB=$PWD/hadoop-bam_amd/lib/variants/libhbam_$v.so; fi
  echo "== $v"
  HBAM_INFLATE_SERIAL=1 HBAM_HUFF_PROF=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 1 --warmup 0 > gpurun_out/x_$v.json 2> gpurun_out/x_$v.err
  grep "lz77 prof" gpurun_out/x_$v.err | head -1
done
exit 0
