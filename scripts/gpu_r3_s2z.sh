#!/bin/bash
# Session 2, call Z: freeze layout + descriptor table cached on the reused
# take plan, module-locality and memory-reading caches on the coalesce path:
# async GPU tests, then bench.py with timelines of the warm async_takes.
set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
O=$PWD/gpurun_out/s2z
mkdir -p $O/tl bench_tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_dlrm_resharding.py -x -v -m gpu \
    -k "async or freeze or kept or drain or hbm or unfrozen" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HIPSNAPSHOT_TIMELINE=$O/tl/b timeout -k 10 300 python bench.py --steps 5 --warmup 2 --async-iters 5 > $O/bench.json 2> $O/bench.err \
    || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
grep async $O/bench.err
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ['value','time_to_unblock_ms','time_to_unblock_ms_each','cold_time_to_unblock_ms','restore_bitwise_ok']})"
rm -rf bench_tmp
