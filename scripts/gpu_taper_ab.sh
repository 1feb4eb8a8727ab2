set -o pipefail
out=gpurun_out/taper_ab; mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p $HIPSNAPSHOT_BENCH_DIR
for i in 1 2; do for m in ${LABELS:-cur}; do
  timeout -k 10 200 python benchmarks/rank_share/main.py --world 1 --steps 8 --warmup 2 --async-iters 1 --restore-iters 1 > $out/w1_${m}_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python benchmarks/rank_share/main.py --world 8 --steps 15 --warmup 3 --async-iters 1 --restore-iters 1 > $out/w8_${m}_$i.json 2>/dev/null || exit 1
  echo "$m $i w1 $(tail -1 $out/w1_${m}_$i.json | cut -c80-200) | w8 $(tail -1 $out/w8_${m}_$i.json | cut -c80-200)"
done; done
