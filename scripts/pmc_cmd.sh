set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INST_LEVEL_LDS --output-format csv -d $R/gpurun_out/pmc1/sq -o run -- python3 $R/scripts/probe_inflate.py 3000000 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $R/gpurun_out/pmc1/ic -o run -- python3 $R/scripts/probe_inflate.py 3000000 >> $R/gpurun_out/pmc1.log 2>&1 || exit 2
