#!/bin/bash
# PMC passes for tools/head_mfma.py (one process per configuration), summary to
# gpurun_out/head_mfma.txt.  Each pass under its own time limit; stop at the
# first pass that does not end normally.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/head_mfma
mkdir -p $OUT
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
# configurations: the script's arguments (e.g. "--m 8192" "--m 16384"), else the round-2 set
if [ $# -gt 0 ]; then CFGS=("$@"); else
  CFGS=("--n 1" "--n 8" "--n 32" "--m 128" "--m 256" "--m 512" "--m 1024" "--m 2048" "--m 4096"); fi
for cfg in "${CFGS[@]}"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -s KILL 120 rocprofv3 --pmc $CTR -d $OUT/$tag -o run --output-format csv -- python3 $R/tools/head_mfma.py $cfg > $OUT/$tag.log 2>&1
  rc=$?
  echo "$cfg rc=$rc" >> $R/gpurun_out/head_mfma.txt
  if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
  f=$(find $OUT/$tag -name "*counter_collection.csv" | head -1)
  echo "== $cfg ($(grep -h 'M=' $OUT/$tag.log | tr '\n' ' '))" >> $R/gpurun_out/head_mfma.txt
  python3 $R/tools/pmc_mfma.py $f >> $R/gpurun_out/head_mfma.txt
done
