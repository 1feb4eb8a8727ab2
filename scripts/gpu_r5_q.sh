#!/bin/bash
# Same-box A/B, HEAD vs f9770d1 (ab_r3/old): DLRM UVM 8 GB save and the DDP 20 GB save.
set -o pipefail
mkdir -p gpurun_out/r5/q
export PYTHONUNBUFFERED=1
for i in ${REPS:-1 2}; do
  for t in ${ORDER:-head old}; do
    if [ $t = head ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/ab_r3/old; fi
    (cd $d && HSBENCH_DIR=/tmp/abq_$t PYTHONPATH=$d timeout -k 10 300 python benchmarks/dlrm_uvm/main.py --total-gb 8 --uvm) > gpurun_out/r5/q/uvm_$t$i.json 2> gpurun_out/r5/q/uvm_$t$i.err || { echo "uvm $t$i failed"; tail -5 gpurun_out/r5/q/uvm_$t$i.err; exit 1; }
    [ -n "$NO_DDP" ] || (cd $d && HSBENCH_DIR=/tmp/abq_$t PYTHONPATH=$d timeout -k 10 300 python benchmarks/ddp/main.py --repeats 3) > gpurun_out/r5/q/ddp_$t$i.json 2> gpurun_out/r5/q/ddp_$t$i.err || { echo "ddp $t$i failed"; tail -5 gpurun_out/r5/q/ddp_$t$i.err; exit 1; }
    rm -rf /tmp/abq_$t
    echo "$t$i uvm $(tail -1 gpurun_out/r5/q/uvm_$t$i.json | grep -o '"sync_GBps": [0-9.]*') ddp $(tail -1 gpurun_out/r5/q/ddp_$t$i.json | grep -o '"GBps": [0-9.]*')"
  done
done
