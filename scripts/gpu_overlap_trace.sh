#!/bin/bash
# Training-step slowdown during an async-take drain, split into launch gaps
# and longer kernels: benchmarks/train_overlap (Llama-3-8B + AdamW) under
# rocprofv3 --kernel-trace, then scripts/overlap_trace_summary.py on the box
# (the raw trace stays in /tmp).  SEQ (default 512), CKPT (3).
set -o pipefail
out=gpurun_out/ovtrace
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HSBENCH_DIR=$PWD/bench_tmp
mkdir -p $HSBENCH_DIR
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
tr=/tmp/ovtrace_$$
SEQ=${SEQ:-512}
timeout -k 10 600 rocprofv3 --kernel-trace ${HIPTRACE:+--hip-runtime-trace} --output-format csv -d $tr -o ov \
    -- python3 benchmarks/train_overlap/main.py --seq $SEQ --checkpoints ${CKPT:-3} \
    --baseline-steps 8 ${ARGS:-} > $out/ov${SEQ}.json 2> $out/ov${SEQ}.err \
    || { echo OV_FAIL; grep -v "^frame" $out/ov${SEQ}.err | tail -30; exit 1; }
tail -1 $out/ov${SEQ}.json
f=$(find $tr -name "*kernel_trace.csv" | head -1)
ls -la $f
timeout -k 10 300 python3 scripts/overlap_trace_summary.py $f --json $out/summary_seq${SEQ}.json \
    > $out/summary_seq${SEQ}.txt || { echo SUM_FAIL; exit 1; }
cat $out/summary_seq${SEQ}.txt
rm -rf $tr
