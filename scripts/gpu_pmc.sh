#!/bin/bash
# Hardware-counter passes (rocprofv3 --pmc) over the data-plane microbench,
# restricted to hipsnapshot's own kernels.  Counter passes use --kernel-trace
# and --stats only (no sys/runtime traces).  Raw CSVs are condensed on the box
# into gpurun_out/pmc_summary.{md,csv} and deleted (they exceed the pull cap).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $REPO/gpurun_out/counters_list.txt 2>&1 || true
dirs=""
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  tag=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --pmc $pass --kernel-include-regex "hs_|hsz_" \
      --output-format csv -d $REPO/gpurun_out/raw_$tag -o pmc -- python3 $REPO/benchmarks/microbench.py --skip-fs \
      > $REPO/gpurun_out/pmc_$tag.log 2>&1 || { echo PMC_FAIL $tag; tail -20 $REPO/gpurun_out/pmc_$tag.log; exit 1; }
  dirs="$dirs $REPO/gpurun_out/raw_$tag"
done
python3 $REPO/scripts/pmc_summary.py $REPO/gpurun_out/pmc_summary $dirs || exit 1
for d in $dirs; do f=$(ls $d/*counter_collection.csv | head -1); head -40 $f > $d.sample.csv; done
rm -rf $dirs
