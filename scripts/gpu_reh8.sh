set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HIPSNAPSHOT_BENCH_DIR=$PWD/bench_tmp
mkdir -p bench_tmp gpurun_out/rehearse
for c in hsz1 none; do
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29811 bench.py --gpus 8 --backend gloo --steps 1 --warmup 1 --async-iters 0 --compression $c > gpurun_out/rehearse/n8_$c.json 2> gpurun_out/rehearse/n8_$c.err || { echo FAIL; grep -v -i "gloo\|^\[W\|amdgpu.ids" gpurun_out/rehearse/n8_$c.err | tail -30; exit 1; }
echo "== $c"; grep -E "^step|^restore|mismatch" gpurun_out/rehearse/n8_$c.err | head -30
done
