set -o pipefail
O=gpurun_out/dropab; mkdir -p $O
for i in 1 2; do
 for v in prev cur; do
  L=hadoop-bam_amd/lib/libhbam.so; [ $v = prev ] && L=hadoop-bam_amd/lib/variants/libhbam_prev.so
  HBAM_LIB=$L timeout -k 10 200 python -u scripts/dropin_probe2.py 10000000 --torch --steps none,none > $O/$v$i.log 2>&1 || { echo "fail $v$i"; tail -20 $O/$v$i.log; exit 3; }
  echo "== $v $i"; grep -E "^(mapped|resident)" $O/$v$i.log | cut -c1-150
 done
done
