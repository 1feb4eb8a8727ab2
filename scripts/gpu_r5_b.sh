#!/bin/bash
# Same-box A/B of the ZeRO-3 save and the DLRM UVM save: HEAD vs the
# round-3 tree (b1de562, extracted into ab_r3/ and built in-tree).
set -o pipefail
R=gpurun_out/r5/b
mkdir -p $R
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
p() { echo "== $*"; timeout -k 10 300 python scripts/probes/zero3_drain_probe.py "$@" >> $R/zero3_ab.jsonl 2>> $R/zero3_ab.err || { echo FAIL; tail -20 $R/zero3_ab.err; exit 1; }; tail -${REP:-2} $R/zero3_ab.jsonl | cut -c1-400; }
p . head
p ab_r3 r3
HIPSNAPSHOT_DRAIN_WRITERS=16 HIPSNAPSHOT_DRAIN_BOOST_WRITERS=16 p . head_w16
HIPSNAPSHOT_DRAIN_WRITERS=16 p ab_r3 r3_w16
HIPSNAPSHOT_DRAIN_WRITERS=16 HIPSNAPSHOT_DRAIN_BOOST_WRITERS=16 HIPSNAPSHOT_DRAIN_NICE=0 HIPSNAPSHOT_DRAIN_AVOID_CALLER_CORE=0 HIPSNAPSHOT_NATIVE_IO_NUMA_LOCAL=0 p . head_w16_plain
run() { name=$1; shift; echo "== $name"; timeout -k 10 420 "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; tail -20 $R/$name.err; exit 1; }; tail -1 $R/$name.json | cut -c1-500; }
run dlrm_uvm_head python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm
run dlrm_uvm_r3 python ab_r3/benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm
run dlrm_uvm_head2 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm
rm -rf $HSBENCH_DIR
