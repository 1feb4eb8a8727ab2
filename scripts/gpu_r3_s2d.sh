#!/bin/bash
# Session 2, call D: DLRM UVM tables never placed / placed in host DRAM /
# placed in HBM (save, async unblock + freeze, restore, bitwise), bench.py.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2d
mkdir -p $O bench_tmp
for pl in default host device; do
  extra=""; [ $pl != default ] && extra="--uvm-place $pl"
  timeout -k 10 300 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm $extra > $O/dlrm_uvm_$pl.json 2> $O/dlrm_uvm_$pl.err \
      || { echo DLRM_FAIL $pl; tail -20 $O/dlrm_uvm_$pl.err; exit 1; }
  tail -1 $O/dlrm_uvm_$pl.json
done
HIPSNAPSHOT_UVM_ASSUME_HOST=0 timeout -k 10 300 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm > $O/dlrm_uvm_default_dma.json 2> $O/dlrm_uvm_default_dma.err \
    || { echo DLRM_FAIL dma; tail -20 $O/dlrm_uvm_default_dma.err; exit 1; }
tail -1 $O/dlrm_uvm_default_dma.json
timeout -k 10 300 python benchmarks/dlrm_uvm/main.py --total-gb 8 > $O/dlrm_hbm.json 2> $O/dlrm_hbm.err \
    || { echo DLRM_FAIL hbm; tail -20 $O/dlrm_hbm.err; exit 1; }
tail -1 $O/dlrm_hbm.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json; grep -E "async" $O/bench.err
df -h /dev/shm /tmp $PWD | cat
free -g | cat
rm -rf bench_tmp
