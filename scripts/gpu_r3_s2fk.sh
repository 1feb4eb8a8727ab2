#!/bin/bash
# Session 2: freeze kernel timing inside async_take; async GPU tests + bench.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2fk
mkdir -p $O bench_tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v -m gpu \
    -k "async or freeze or kept or drain or hbm or unfrozen" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['value','time_to_unblock_ms','cold_time_to_unblock_ms','freeze_gpu_ms','freeze_kernel_ms','unblock_incl_freeze_ms','async_total_ms','restore_GBps','restore_bitwise_ok','raw_GBps','fresh_path_GBps','ddp20gb_fp32_s']})"
rm -rf bench_tmp
