#!/bin/bash
# Config 4 at the W=8 share: 12.5 GB of UVM tables, 7 host siblings.
set -o pipefail
R=gpurun_out/r5/h
mkdir -p $R
export PYTHONUNBUFFERED=1 HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
df -h $HSBENCH_DIR /dev/shm /tmp 2>&1 | tee $R/df.txt
free -g | tee $R/free.txt
run() { name=$1; shift; echo "== $name"; timeout -k 10 ${T:-500} "$@" > $R/$name.json 2> $R/$name.err || { echo "FAIL $name"; grep -v "^frame" $R/$name.err | tail -20; exit 1; }; tail -1 $R/$name.json | cut -c1-1500; }
# siblings write to /dev/shm when the bench disk cannot hold 8 ranks' blobs
avail=$(df -k --output=avail $HSBENCH_DIR | tail -1)
if [ $avail -lt 130000000 ]; then export HSBENCH_SIBLING_DIR=/dev/shm/hs_sib; echo "siblings -> /dev/shm"; fi
T=600 run dlrm_uvm_w8share_solo python benchmarks/dlrm_uvm/main.py --total-gb 12.5 --uvm --single-path
T=600 run dlrm_uvm_w8share_sib7 python benchmarks/dlrm_uvm/main.py --total-gb 12.5 --uvm --single-path --host-siblings 7
rm -rf $HSBENCH_DIR /dev/shm/hs_sib
