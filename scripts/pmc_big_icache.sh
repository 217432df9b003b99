# SQ / SQC counters of the workgroup kernel on 512 configs[4] reactors (scripts/c5_once.py), one
# rocprofv3 pass per line.  Usage: pmc_big_icache.sh [TAG]
set -o pipefail
TAG=${1:-r05ic}
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- python3 scripts/c5_once.py 512 > gpurun_out/pmc_${TAG}_p$i.log 2>&1
  rc=$?
  tail -1 gpurun_out/pmc_${TAG}_p$i.log
  if [ $rc -ne 0 ]; then echo "pass $i status $rc: stop"; exit $rc; fi
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH
SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_MFMA_F64
SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES
LIST
python3 scripts/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/pmc_${TAG}_summary.txt 2>&1; cat gpurun_out/pmc_${TAG}_summary.txt
